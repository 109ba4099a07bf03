"""Find software-pipelined loops whose first vmcnt wait at the loop head also waits for
stores issued at the end of the previous iteration: for every backward
branch in a kernel's ISA, the loop body's trailing stores (after its last load) are
counted and compared with the first `s_waitcnt vmcnt(n)` after the loop head.

    cd /tmp/asm && hipcc --offload-arch=gfx950 -O3 -std=c++17 -I/root/repo/include \
        --save-temps -c -o x.o /root/repo/ska-pst-dsp-model_amd/csrc/pfb_analysis.hip
    python scripts/isa_loop_waits.py /tmp/asm/*gfx950.s
"""
import sys,re,glob
def funcs(txt):
    for m in re.finditer(r'^(_Z\w+):[^\n]*\n(.*?)\.Lfunc_end', txt, re.S|re.M):
        yield m.group(1), m.group(2).split('\n')
for f in sys.argv[1:]:
    txt=open(f).read()
    for name, lines in funcs(txt):
        ins=[l.split(';')[0].strip() for l in lines]
        ins=[l for l in ins if l]
        labels={l[:-1]:i for i,l in enumerate(ins) if l.endswith(':')}
        for i,l in enumerate(ins):
            m=re.match(r's_cbranch_\w+ (\.LBB\w+)|s_branch (\.LBB\w+)', l)
            if not m: continue
            tgt=m.group(1) or m.group(2)
            h=labels.get(tgt)
            if h is None or h>i: continue
            body=ins[h:i+1]
            # trailing stores: count vmem ops after last load in body (in order)
            vm=[('L' if re.match(r'(buffer|global)_load',x) else 'S') for x in body if re.match(r'(buffer|global)_(load|store)',x)]
            if 'S' not in vm: continue
            trail=0
            for x in reversed(vm):
                if x=='S': trail+=1
                else: break
            # first vmcnt wait after head, before any vmem op
            first=None
            for x in body:
                if re.match(r'(buffer|global)_(load|store)',x): break
                mm=re.search(r'vmcnt\((\d+)\)',x)
                if mm: first=int(mm.group(1)); break
            if first is not None and first < trail:
                print(f"{name[:90]}  head {tgt}: first wait vmcnt({first}) < {trail} trailing stores")
