"""Per-kernel mean of rocprofv3 --pmc counters (counter_collection.csv) for kernels matching a pattern,
plus the derived ratios used in profiles/README.md."""
import collections
import csv
import sys


def main(paths, pat):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in paths:
        for r in csv.DictReader(open(path)):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
            if pat not in k:
                continue
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in agg.items():
        m = {c: sum(v) / len(v) for c, v in d.items()}
        row = {c: f"{v:.4g}" for c, v in m.items()}
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_LDS"):
                if c in m:
                    row[c + "/WAVE"] = f"{m[c] / wc:.3f}"
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "GRBM_GUI_ACTIVE" in m:
            row["MFMA_util"] = f"{m['SQ_VALU_MFMA_BUSY_CYCLES'] / (m['GRBM_GUI_ACTIVE'] * 256 * 4):.3f}"
        print(k, row)


if __name__ == "__main__":
    main(sys.argv[2:], sys.argv[1])
