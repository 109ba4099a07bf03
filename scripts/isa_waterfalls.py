"""Count one-trip waterfall loops per kernel in a gfx950 ISA listing: a `v_readfirstlane`
followed within a few instructions by `s_and_saveexec` and a buffer / global access — the
form the compiler emits when a buffer descriptor or scalar offset lives in a VGPR
(DESIGN.md §11).

    cd /tmp/asm && hipcc --offload-arch=gfx950 -O3 -std=c++17 -I/root/repo/include \\
        --save-temps -c -o x.o /root/repo/ska-pst-dsp-model_amd/csrc/pfb_rowfft.hip
    python scripts/isa_waterfalls.py /tmp/asm/*gfx950.s
"""
import re
import sys


def main(paths):
    for f in paths:
        lines = open(f).read().split("\n")
        name, res = None, {}
        for i, l in enumerate(lines):
            if re.match(r"^_Z\w+:", l):
                name = l.split(":")[0]
                continue
            if "v_readfirstlane_b32" in l and name:
                nxt = " ".join(lines[i + 1:i + 12])
                if "s_and_saveexec" in nxt and ("buffer_" in nxt or "global_" in nxt):
                    res[name] = res.get(name, 0) + 1
        for k, v in res.items():
            print(f"{v:4d} {k[:110]}")


if __name__ == "__main__":
    main(sys.argv[1:])
