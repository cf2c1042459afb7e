"""Sum rocprofv3 --pmc counter_collection.csv files per kernel (tools/pmc_cmd.sh output).

python tools/pmc_summarize.py gpurun_out/pmc_s5 > profiles/<name>.txt
"""
from __future__ import annotations

import csv
import glob
import os
import sys
from collections import defaultdict


def main(root: str) -> None:
    vals: dict[str, dict[str, float]] = defaultdict(lambda: defaultdict(float))
    disp: dict[str, dict[str, set]] = defaultdict(lambda: defaultdict(set))
    for f in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
        with open(f, newline="") as fh:
            for r in csv.DictReader(fh):
                k = r["Kernel_Name"].split("(")[0]
                vals[k][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[k][f].add(r["Dispatch_Id"])
    order = sorted(vals, key=lambda k: -vals[k].get("SQ_BUSY_CU_CYCLES", 0.0))
    names = sorted({c for v in vals.values() for c in v})
    print("# per-kernel counter sums over all dispatches of the profiled run")
    print("# derived: mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / SQ_BUSY_CU_CYCLES; l2_hit = HIT / (HIT + MISS)")
    for k in order:
        v = vals[k]
        line = [f"{k[:90]:90s} dispatches={max(len(d) for d in disp[k].values())}"]
        busy = v.get("SQ_BUSY_CU_CYCLES", 0.0)
        if busy:
            line.append(f"mfma_busy={v.get('SQ_VALU_MFMA_BUSY_CYCLES', 0.0) / busy:.3f}")
        hm = v.get("TCC_HIT_sum", 0.0) + v.get("TCC_MISS_sum", 0.0)
        if hm:
            line.append(f"l2_hit={v.get('TCC_HIT_sum', 0.0) / hm:.3f}")
        print("  ".join(line))
        print("    " + "  ".join(f"{c}={v[c]:.4g}" for c in names if c in v))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_s5")
