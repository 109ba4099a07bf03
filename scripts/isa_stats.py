"""Per-kernel VGPR / AGPR / LDS / occupancy summary of a hipcc --save-temps gfx950 .s file."""
import re
import sys

VALU = re.compile(r"^\s+v_", re.M)
DS = re.compile(r"^\s+ds_", re.M)
txt = open(sys.argv[1]).read()
flt = sys.argv[2] if len(sys.argv) > 2 else ""
for m in re.finditer(r"^(_Z\S+):[^\n]*\n(.*?)^\s*s_endpgm", txt, re.S | re.M):
    name = m.group(1)
    tail = txt[m.end(): m.end() + 3000]

    def g(k):
        r = re.search(rf"; {k}: (\d+)", tail)
        return r.group(1) if r else "?"

    if flt in name:
        body = m.group(2)
        nv, nd = len(VALU.findall(body)), len(DS.findall(body))
        print(f"{name[:100]:100s} vgpr={g('NumVgprs')} agpr={g('NumAgprs')} lds={g('LDSByteSize')} "
              f"occ={g('Occupancy')} scratch={g('ScratchSize')} pkfma={body.count('v_pk_fma_f32')} "
              f"valu={nv} ds={nd}")
