"""Check a hipcc -S listing for values read from the fused rows' clobbered temporaries
(v6-v11) after a fused-row asm block without being rewritten first (mont27_fused_gen.h).

    python tools/clobcheck.py listing.s KERNEL_MANGLED_SUBSTRING..."""
import re,sys
def regs(op):
    out=set()
    for m in re.finditer(r'v\[(\d+):(\d+)\]|\bv(\d+)\b',op):
        if m.group(3): out.add(int(m.group(3)))
        else: out.update(range(int(m.group(1)),int(m.group(2))+1))
    return out
def check(f,kname,watch=range(6,12)):
    L=open(f).read().split('\n');out=[];on=False
    for l in L:
        if re.match(r'^_Z\w*'+kname+r'\w*:',l): on=True;continue
        if on and l.strip().startswith('.Lfunc_end'): break
        if on: out.append(l.strip())
    bad=0; nblk=0
    i=0
    while i<len(out):
        if out[i].startswith(';;#ASMSTART'):
            j=i
            while not out[j].startswith(';;#ASMEND'): j+=1
            body=' '.join(out[i:j])
            if 'v_and_b32_dpp v11' in body:
                nblk+=1
                live=set(watch)
                k=j+1
                while k<len(out) and live and k<j+400:
                    s=out[k]
                    if s.startswith(';;#ASMSTART'):
                        # a later fused block redefines v6-v11 before use
                        break
                    if s and not s.startswith(';') and not s.startswith('.') and not s.endswith(':'):
                        parts=s.split(None,1)
                        if len(parts)>1:
                            ops=[o.strip() for o in parts[1].split(',')]
                            op=parts[0]
                            is_store=op.startswith(('buffer_store','scratch_store','global_store','ds_write','flat_store'))
                            dst=set() if is_store else regs(ops[0])
                            src=regs(','.join(ops if is_store else ops[1:]))
                            r=src & live
                            if r:
                                bad+=1; print('READ-after-asm', sorted(r), 'line', k, s); live-=r
                            live-=dst
                    if s.startswith('s_branch') or s.startswith('s_cbranch') or s.startswith('s_setpc') : break
                    k+=1
            i=j
        i+=1
    print(kname, 'fused blocks', nblk, 'violations', bad)
for k in sys.argv[2:]: check(sys.argv[1],k)
