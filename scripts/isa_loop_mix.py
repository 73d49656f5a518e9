"""Instruction mix of the loops of one kernel in a device assembly file (hipcc --cuda-device-only -S).

    python scripts/isa_loop_mix.py attn.s attn_fwd_kernelILb1ELi2ELi4ELi4

A loop is a label that a later s_cbranch / s_branch in the same function jumps back to; the body is
every instruction between the label and that branch.  Classes: MFMA, VALU (with transcendental
v_exp / v_log / v_rcp / v_rsq / v_sqrt counted separately), DS reads / writes, VMEM, SALU, waits.
"""
import re
import sys


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith(("v_exp", "v_log", "v_rcp", "v_rsq", "v_sqrt", "v_sin", "v_cos")):
        return "trans"
    if op.startswith("v_permlane"):
        return "permlane"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_read") or op.startswith("ds_load"):
        return "ds_read"
    if op.startswith("ds_"):
        return "ds_write"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_barrier"):
        return "barrier"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    path, name = sys.argv[1], sys.argv[2]
    lines = open(path).read().splitlines()
    start = next(i for i, ln in enumerate(lines) if re.match(rf"^\S*{name}\S*:", ln))
    end = next((i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end")), len(lines))
    body = lines[start:end]
    labels = {}
    for i, ln in enumerate(body):
        m = re.match(r"^(\.LBB\w+):", ln)
        if m:
            labels[m.group(1)] = i
    for i, ln in enumerate(body):
        m = re.match(r"^\s+s_(cbranch_\w+|branch)\s+(\.LBB\w+)", ln)
        if m and m.group(2) in labels and labels[m.group(2)] < i:
            lo = labels[m.group(2)]
            mix = {}
            for b in body[lo:i + 1]:
                t = b.strip()
                if not t or t.startswith((";", ".")) or t.endswith(":"):
                    continue
                c = classify(t.split()[0])
                mix[c] = mix.get(c, 0) + 1
            print(f"loop {m.group(2)} lines {lo}-{i}: " + ", ".join(f"{k} {v}" for k, v in sorted(mix.items())))


if __name__ == "__main__":
    main()
