"""Condensed ISA listing of one kernel: barriers, memory instructions, branches, labels
and vmcnt waits, with the VALU/DS instructions between them counted.

    python scripts/isa_wait_listing.py kernel-gfx950.s <mangled kernel name>
"""
import sys
txt=open(sys.argv[1]).read()
name=sys.argv[2]
i=txt.index(name+':'); j=txt.index('.Lfunc_end',i)
body=txt[i:j].split('\n')
cnt=0; out=[]
for ln in body:
    s=ln.split(";")[0].strip()
    if not s or s.startswith(';') or (s.startswith('.') and not s.endswith(':')): continue
    op=s.split()[0]
    if op.startswith(('v_','ds_')): cnt+=1; continue
    if op.startswith(('s_barrier','buffer_','global_','s_cbranch','s_branch','s_endpgm')) or ('vmcnt' in s) or s.endswith(':'):
        if cnt: out.append(f"   [{cnt} valu/ds]"); cnt=0
        out.append(s[:90])
print('\n'.join(out))
