#!/usr/bin/env python3
"""Static instruction budget of a kernel's main loop from hipcc -S output (make asm SRC=...):
per function, the largest loop body (a label ... backward branch to it) split by instruction
class. Usage: python tools/isa_count.py /tmp/k_front3.hip.s [substring of the kernel symbol]"""
import re
import sys
from collections import Counter


def functions(lines):
    cur, body = None, []
    for ln in lines:
        m = re.match(r'^(_Z\S+):\s*(;.*)?$', ln)
        if m:
            if cur:
                yield cur, body
            cur, body = m.group(1), []
        elif cur:
            if ln.startswith('.Lfunc_end'):
                yield cur, body
                cur, body = None, []
            else:
                body.append(ln)


def klass(op):
    if op.startswith('v_mfma'):
        return 'mfma'
    if op.startswith(('v_pk_fma', 'v_pk_mul', 'v_pk_add')):
        return 'valu_pk_f32'
    if op.startswith(('v_fma', 'v_fmac', 'v_mul_f', 'v_add_f', 'v_sub_f', 'v_subrev_f', 'v_mac_f')):
        return 'valu_f32_arith'
    if op.startswith(('v_dot2', 'v_perm', 'v_cvt')):
        return 'valu_' + op.split('_')[1]
    if op.startswith(('v_mov_b32_dpp', 'v_permlane')) or '_dpp' in op:
        return 'valu_xlane'
    if op.startswith(('v_mov', 'v_cndmask')):
        return 'valu_mov'
    if op.startswith('v_'):
        return 'valu_other'
    if op.startswith('ds_read') or op.startswith('ds_load'):
        return 'lds_read'
    if op.startswith('ds_write') or op.startswith('ds_store'):
        return 'lds_write'
    if op.startswith(('global_load', 'buffer_load', 'flat_load')):
        return 'vmem_load'
    if op.startswith(('global_store', 'buffer_store', 'flat_store')):
        return 'vmem_store'
    if op.startswith('s_waitcnt'):
        return 'waitcnt'
    if op.startswith('s_barrier'):
        return 'barrier'
    if op.startswith('s_'):
        return 'salu'
    return 'other'


def main():
    path = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else ''
    lines = open(path).read().splitlines()
    for name, body in functions(lines):
        if pat not in name:
            continue
        labels = {}
        spans = []
        for i, ln in enumerate(body):
            m = re.match(r'^(\.LBB\d+_\d+):', ln)
            if m:
                labels[m.group(1)] = i
            m = re.search(r'\ts_cbranch_\w+\s+(\.LBB\d+_\d+)', ln) or re.search(r'\ts_branch\s+(\.LBB\d+_\d+)', ln)
            if m and m.group(1) in labels and labels[m.group(1)] < i:
                spans.append((labels[m.group(1)], i))
        # outermost loops, largest first (k_front3 has one per wave role)
        spans.sort(key=lambda sp: sp[0] - sp[1])
        outer = []
        for sp in spans:
            if not any(o[0] <= sp[0] and sp[1] <= o[1] for o in outer):
                outer.append(sp)
        for best in outer[:int(sys.argv[3]) if len(sys.argv) > 3 else 1]:
            report(name, body, best)


def report(name, body, best):
    if True:
        cnt = Counter()
        for ln in body[best[0]:best[1] + 1]:
            s = ln.strip()
            if not s or s.startswith(('.', ';')) or s.endswith(':'):
                continue
            cnt[klass(s.split()[0])] += 1
        valu = sum(v for k, v in cnt.items() if k.startswith('valu'))
        print(name[:90])
        print('  loop lines %d-%d: VALU %d' % (best[0], best[1], valu))
        for k, v in sorted(cnt.items(), key=lambda kv: -kv[1]):
            print('    %-16s %5d' % (k, v))


if __name__ == '__main__':
    main()
