"""Per-kernel roofline table of one training step from rocprofv3 ``--kernel-trace --pmc`` CSV passes.

Each pass directory holds ``*_kernel_trace.csv`` (dispatch durations) and ``*_counter_collection.csv``
(counters per dispatch); the passes run the same program, so kernels are matched by name and the
per-dispatch means are combined.  Columns: share of kernel time, mean us per dispatch, TFLOP/s from
the MFMA count (every dispatch's SQ_INSTS_MFMA x FLOP per MFMA of the kernel's shape), MFMA-pipe busy
share of all SIMD cycles (SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x duration x clock)), HBM-side
traffic (FETCH_SIZE + WRITE_SIZE, KiB in rocprofv3's units) and its rate, and LDS bank-conflict cycles
per LDS instruction.

usage: python scripts/step_roofline.py PASS_DIR [PASS_DIR ...] [--top 25] [--flop_per_mfma 16384]
"""
import argparse
import collections
import csv
import glob
import os


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    if name.startswith("void "):
        name = name[5:]
    return name.split("(")[0][:72]


def load(dirs):
    dur = collections.defaultdict(list)
    ctr = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in dirs:
        for path in glob.glob(os.path.join(d, "**", "*_kernel_trace.csv"), recursive=True):
            for r in csv.DictReader(open(path)):
                dur[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        for path in glob.glob(os.path.join(d, "**", "*_counter_collection.csv"), recursive=True):
            per = collections.defaultdict(float)
            names = {}
            for r in csv.DictReader(open(path)):
                key = (r.get("Dispatch_Id") or r.get("Correlation_Id"), r["Counter_Name"])
                per[key] += float(r["Counter_Value"])  # summed over XCDs / instances
                names[key[0]] = short(r["Kernel_Name"])
            for (disp, cname), v in per.items():
                ctr[names[disp]][cname].append(v)
    return dur, ctr


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--clock_ghz", type=float, default=None,
                    help="clock for the MFMA-busy share (default: GRBM_GUI_ACTIVE / 8 XCDs / duration)")
    args = ap.parse_args()
    dur, ctr = load(args.dirs)
    # kernel time from the trace of the first pass only (every pass runs the same dispatches)
    first = collections.defaultdict(list)
    for path in glob.glob(os.path.join(args.dirs[0], "**", "*_kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            first[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    total = sum(sum(v) for v in first.values())
    rows = sorted(first.items(), key=lambda kv: -sum(kv[1]))[: args.top]
    print(f"{'share':>6} {'us/call':>9} {'calls':>5} {'TF/s':>7} {'MFMA%':>6} {'clkGHz':>6} {'HBM GB':>7} {'TB/s':>5} "
          f"{'confl/LDS':>9}  kernel")
    for name, ds in rows:
        us = sum(ds) / len(ds)
        c = {k: sum(v) / len(v) for k, v in ctr.get(name, {}).items()}
        mf = c.get("SQ_INSTS_MFMA")
        flop_per = 32768 if "attn" in name else 16384  # 32x32x16 vs 16x16x32 bf16 (x2 FLOP per MAC)
        tf = mf * flop_per / (us * 1e-6) / 1e12 if mf else float("nan")
        gui = c.get("GRBM_GUI_ACTIVE")
        clk = args.clock_ghz or (gui / 8 / (us * 1e3) if gui else float("nan"))
        busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES")
        mfma_pct = 100 * busy / (1024 * us * 1e3 * clk) if busy and clk == clk else float("nan")
        fetch, write = c.get("FETCH_SIZE"), c.get("WRITE_SIZE")
        gb = ((fetch or 0) + (write or 0)) * 1024 / 1e9 if (fetch or write) else float("nan")
        tbs = gb / (us * 1e-6) / 1e3 if gb == gb else float("nan")
        lds, conf = c.get("SQ_INSTS_LDS"), c.get("SQ_LDS_BANK_CONFLICT")
        cpl = conf / lds if lds else float("nan")
        print(f"{100 * sum(ds) / total:6.2f} {us:9.1f} {len(ds):5d} {tf:7.1f} {mfma_pct:6.1f} {clk:6.2f} {gb:7.2f} "
              f"{tbs:5.2f} {cpl:9.3f}  {name}")


if __name__ == "__main__":
    main()
