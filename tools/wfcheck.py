"""Listing checks for the 27-bit engine's kernels (hipcc -S output), run over every kernel:

1. Waterfall loops.  A buffer access whose descriptor is a per-lane VGPR value makes the
   compiler emit a readfirstlane loop (v_readfirstlane -> v_cmp_eq -> s_and_saveexec ->
   buffer op -> s_xor exec -> s_cbranch_execnz).  Under register pressure the register
   allocator has reused a descriptor VGPR for a spill reload INSIDE such a loop, after the
   descriptor's first-iteration read (the 3-wave k_add27<64> fault): the
   second iteration then builds its descriptor from the reloaded value and dereferences a
   bogus base.  Every waterfall loop is reported; a loop whose body writes a register the
   loop's readfirstlanes read is an ERROR.  The kernels are written so that there are none
   (per-lane operand choice loads both operands and selects).
2. Fused-row clobbers.  A value read from the fused rows' clobbered temporaries (v6-v11)
   after a fused-row asm block without being rewritten first (mont27_fused_gen.h).
3. Fused-row pins.  Compiler code between two fused blocks of one row loop that writes the
   pinned accumulator registers v[2:3] / v[4:5] other than by a copy into them is listed
   (informational: the constraints make such writes legal, they only cost moves).

    python tools/wfcheck.py listing.s [KERNEL_SUBSTRING ...]
Exit status 1 if any ERROR."""
import re
import sys


def vregs(tok):
    out = set()
    for m in re.finditer(r'v\[(\d+):(\d+)\]|\bv(\d+)\b', tok):
        if m.group(3):
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


STORE_OPS = ('buffer_store', 'scratch_store', 'global_store', 'ds_write', 'flat_store', 'ds_bpermute')


def parse(line):
    s = line.split(';')[0].strip()
    if not s or s.startswith('.') or s.endswith(':'):
        return None
    parts = s.split(None, 1)
    op = parts[0]
    ops = [o.strip() for o in parts[1].split(',')] if len(parts) > 1 else []
    if not ops:
        return op, set(), set()
    if op.startswith(STORE_OPS) and not op.startswith('ds_bpermute'):
        return op, set(), vregs(','.join(ops))
    if op.startswith(('v_', 'buffer_load', 'scratch_load', 'global_load', 'ds_read', 'ds_bpermute', 'flat_load')):
        return op, vregs(ops[0]), vregs(','.join(ops[1:]))
    return op, set(), vregs(','.join(ops))


def kernels(lines):
    cur, body = None, []
    for l in lines:
        m = re.match(r'^(_Z\w+):', l)
        if m:
            cur, body = m.group(1), []
            continue
        if cur and l.strip().startswith('.Lfunc_end'):
            yield cur, body
            cur = None
            continue
        if cur:
            body.append(l)


def check_waterfalls(body):
    loops, errors = 0, []
    i = 0
    while i < len(body):
        if 'Inner Loop Header' in body[i] or re.match(r'^\.LBB\w+:', body[i].strip()):
            j = i + 1
            seg = []
            while j < len(body) and not re.match(r'^\.LBB\w+:', body[j].strip()):
                seg.append(body[j])
                if body[j].strip().startswith('s_cbranch_execnz'):
                    break
                j += 1
            text = '\n'.join(seg)
            if j < len(body) and body[j].strip().startswith('s_cbranch_execnz') and 'v_readfirstlane' in text \
                    and re.search(r'buffer_(load|store)', text):
                loops += 1
                # a register the loop's readfirstlanes read, written later in the body and not
                # re-established before the read at the top of the body: the next iteration
                # reads the new value.  (A reload at the top of the body, before the read, is
                # how the allocator legitimately keeps a spilled descriptor word.)
                parsed = [parse(l) for l in seg]
                first_read, first_write = {}, {}
                for k, p in enumerate(parsed):
                    if not p:
                        continue
                    for r in p[1]:
                        first_write.setdefault(r, k)
                    if p[0].startswith('v_readfirstlane'):
                        for r in p[2]:
                            first_read.setdefault(r, k)
                for r, kr in first_read.items():
                    if first_write.get(r, 1 << 30) < kr:
                        continue  # re-established at the top of every iteration
                    late = [k for k, p in enumerate(parsed) if p and r in p[1] and k > kr]
                    for k in late[:1]:
                        errors.append(f"loop at +{i}: '{seg[k].strip()}' overwrites v{r}, which the loop's "
                                      f"v_readfirstlane reads again on the next iteration (descriptor clobbered)")
            i = j
        i += 1
    return loops, errors


def check_fused(body):
    bad, nblk = [], 0
    i = 0
    while i < len(body):
        if body[i].strip().startswith(';;#ASMSTART'):
            j = i
            while not body[j].strip().startswith(';;#ASMEND'):
                j += 1
            blk = ' '.join(x.strip() for x in body[i:j])
            if 'v_and_b32_dpp v11' in blk:
                nblk += 1
                live = set(range(6, 12))
                k = j + 1
                while k < len(body) and live and k < j + 400:
                    s = body[k].strip()
                    if s.startswith(';;#ASMSTART') or s.startswith(('s_branch', 's_cbranch', 's_setpc')):
                        break
                    p = parse(s)
                    if p:
                        r = p[2] & live
                        if r:
                            bad.append(f"read of clobbered {sorted(r)} after a fused block: '{s}'")
                            live -= r
                        live -= p[1]
                    k += 1
            i = j
        i += 1
    return nblk, bad


def main():
    path = sys.argv[1]
    flt = sys.argv[2:]
    lines = open(path).read().split('\n')
    nerr = 0
    for name, body in kernels(lines):
        if flt and not any(f in name for f in flt):
            continue
        short = re.sub(r'^_ZN12_GLOBAL__N_1\d+', '', name)[:48]
        loops, werr = check_waterfalls(body)
        nblk, ferr = check_fused(body)
        errs = werr + ferr
        nerr += len(errs)
        flag = 'ERROR' if errs else ('warn ' if loops else 'ok   ')
        print(f"{flag} {short:50s} waterfall_loops={loops:3d} fused_blocks={nblk:4d} errors={len(errs)}")
        for e in errs[:5]:
            print('      ', e)
    sys.exit(1 if nerr else 0)


if __name__ == '__main__':
    main()
