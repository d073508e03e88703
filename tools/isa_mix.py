#!/usr/bin/env python3
"""Instruction mix of one kernel in a hipcc -S listing (design tool, round 4): resource counts and
a per-class histogram of the basic blocks with >= MIN instructions.

    python3 tools/isa_mix.py lc.s _ZN4jaad16lc_decode_kernelILi0ELi0ELb1EEEvNS_10KernelArgsE [MIN]
"""
import collections
import re
import sys


def classify(k: str) -> str:
    if k.startswith("v_pk_"):
        return "vpk"
    if k.startswith("v_cndmask") and k.endswith("_e32") or k.startswith("v_cndmask_b32_dpp"):
        return "CNDMASK_VCC"
    if k.startswith("v_cndmask"):
        return "cndmask_e64"
    if "_dpp" in k:
        return "dpp"
    if k.startswith("v_permlane"):
        return "permlane"
    if k in ("v_addc_co_u32_e32", "v_add_co_u32_e32", "v_subb_co_u32_e32", "v_sub_co_u32_e32"):
        return "VCC_CARRY"
    if k.startswith("v_"):
        return "valu"
    if k.startswith("ds_"):
        return "lds"
    if k.startswith(("global_", "buffer_")):
        return "vmem"
    if k.startswith("s_waitcnt"):
        return "waitcnt"
    if k.startswith("s_nop"):
        return "nop"
    if k.startswith("s_"):
        return "salu"
    return k


def main():
    path, name = sys.argv[1], sys.argv[2]
    mn = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    s = open(path).read().split("\n")
    start = [i for i, l in enumerate(s) if l.startswith(name + ":")][0]
    end = [i for i in range(start, len(s)) if s[i].strip().startswith("s_endpgm")][0]
    blocks, cur, lab = [], [], "entry"
    for l in s[start:end + 1]:
        m = re.match(r"^(\.LBB\w+):", l)
        if m:
            blocks.append((lab, cur))
            lab, cur = m.group(1), []
            continue
        t = l.strip()
        if t and not t.startswith((";", ".")):
            cur.append(t.split()[0])
    blocks.append((lab, cur))
    meta = "\n".join(s[end:end + 400])
    for key in ("vgpr_count", "sgpr_count", "vgpr_spill_count", "group_segment_fixed_size"):
        m = re.search(rf"\.{key}:\s+(\d+)", "\n".join(s[end:]).split(".name:")[0] if False else meta)
    # resource lines printed by the compiler after the kernel
    tail = "\n".join(s[end:end + 60])
    for key in ("NumVgprs", "NumSgprs", "ScratchSize", "Occupancy", "LDSByteSize"):
        m = re.search(rf"; {key}: (\d+)", tail)
        if m:
            print(f"{key}: {m.group(1)}")
    tot = collections.Counter()
    for lab, ins in blocks:
        c = collections.Counter(classify(k) for k in ins)
        tot += c
        if len(ins) >= mn:
            print(lab, len(ins), dict(sorted(c.items(), key=lambda x: -x[1])))
    print("static total", sum(tot.values()), dict(sorted(tot.items(), key=lambda x: -x[1])))


if __name__ == "__main__":
    main()
