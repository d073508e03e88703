"""Rough VGPR liveness over an AMDGPU .s function: prints the peak live count and what is live there.

usage: python tools/vgpr_live.py file.s kernel_symbol [n_context]
Heuristic def/use rules (first VGPR operand is the def for instructions that write a VGPR);
good enough to find which values keep the register pressure up."""
import re
import sys
from collections import defaultdict

REG = re.compile(r'\bv\[(\d+):(\d+)\]|\bv(\d+)\b')


def regs(tok):
    out = set()
    for m in REG.finditer(tok):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


NO_DEF = ('ds_write', 'global_store', 'buffer_store', 'scratch_store', 'flat_store', 'v_cmp', 'v_cmpx',
          'v_readlane', 'v_readfirstlane', 'ds_bpermute_dummy', 's_', 'exp ')
RMW = ('v_writelane', 'v_mac', 'v_fmac', 'v_swap', 'v_cndmask_dummy')


def main():
    path, sym = sys.argv[1], sys.argv[2]
    nctx = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    lines = open(path).read().split('\n')
    start = next(i for i, l in enumerate(lines) if l.startswith(sym + ':'))
    body = []
    for l in lines[start + 1:]:
        if '.end_amdhsa_kernel' in l or l.startswith('.Lfunc_end'):
            break
        body.append(l)
    insts, labels = [], {}
    for l in body:
        t = l.split(';')[0].strip()
        if not t:
            continue
        if t.endswith(':'):
            labels[t[:-1]] = len(insts)
            continue
        if t.startswith('.'):
            continue
        insts.append(t)
    n = len(insts)
    defs, uses, succ = [], [], []
    for i, t in enumerate(insts):
        op = t.split()[0]
        rest = t[len(op):]
        ops = [o.strip() for o in rest.split(',')] if rest.strip() else []
        d, u = set(), set()
        if ops:
            first = regs(ops[0])
            others = set()
            for o in ops[1:]:
                others |= regs(o)
            if op.startswith(NO_DEF) or not first:
                u = first | others
            else:
                d = first
                u = others
                if op.startswith(RMW) or '_sdwa' in op or 'd16_hi' in op or 'd16' in op:
                    u |= first
        defs.append(d)
        uses.append(u)
        s = []
        if op == 's_branch':
            s = [labels[ops[0]]]
        elif op.startswith('s_cbranch'):
            s = [labels[ops[0]], i + 1]
        elif op in ('s_endpgm', 's_setpc_b64'):
            s = []
        else:
            s = [i + 1]
        succ.append([x for x in s if x < n])
    live_in = [set() for _ in range(n)]
    changed = True
    while changed:
        changed = False
        for i in range(n - 1, -1, -1):
            lo = set()
            for s in succ[i]:
                lo |= live_in[s]
            li = (lo - defs[i]) | uses[i]
            if li != live_in[i]:
                live_in[i] = li
                changed = True
    lo_i = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    hi_i = int(sys.argv[5]) if len(sys.argv) > 5 else n
    prof = [max(len(live_in[j]) for j in range(i, min(n, i + 250))) for i in range(0, n, 250)]
    print('profile (max live per 250 instructions):', prof)
    peak = max(range(lo_i, hi_i), key=lambda i: len(live_in[i]))
    print(f'{n} instructions, peak live VGPRs {len(live_in[peak])} at #{peak}: {insts[peak]}')
    hist = sorted(((len(live_in[i]), i) for i in range(n)), reverse=True)[:5]
    print('top points:', [(c, i) for c, i in hist])
    if nctx:
        for i in range(max(0, peak - nctx), min(n, peak + nctx)):
            print(f'{i:6d} {len(live_in[i]):4d}  {insts[i]}')
    # for every register live at the peak: the next instruction (in layout order, wrapping) that reads it
    if len(sys.argv) > 6:
        for r in sorted(live_in[peak]):
            nxt = next((j for j in list(range(peak, n)) + list(range(0, peak)) if r in uses[j]), None)
            print(f'  v{r:<4d} next use #{nxt}: {insts[nxt] if nxt is not None else "-"}'[:130])
    # live ranges spanning the peak: where each live register was last defined before it
    lastdef = {}
    for i in range(peak):
        for r in defs[i]:
            lastdef[r] = i
    print('live at peak, grouped by defining instruction:')
    by = defaultdict(list)
    for r in sorted(live_in[peak]):
        by[lastdef.get(r, -1)].append(r)
    for i in sorted(by):
        print(f'  def #{i:6d} {insts[i] if i >= 0 else "(loop-carried/entry)"[:90]:90.90s} -> {len(by[i])} regs')


if __name__ == '__main__':
    main()
