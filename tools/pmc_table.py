#!/usr/bin/env python
"""Per-kernel PMC table from tools/pmc_head.sh output (medians per dispatch):

    python tools/pmc_table.py gpurun_out/pmc/<case> > profiles/<name>.txt

mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (4 * SQ_BUSY_CU_CYCLES) (4 SIMDs per CU; indicative, for ranking);
l2_hit = TCC_HIT / (HIT + MISS); wait = SQ_WAIT_ANY / SQ_WAVE_CYCLES; lds_conf = SQ_LDS_BANK_CONFLICT /
SQ_LDS_IDX_ACTIVE (share of LDS cycles lost to bank conflicts); VALU/MFMA = instruction ratio.
"""
from __future__ import annotations

import csv
import glob
import statistics
import sys
from collections import defaultdict


def main(prefix: str) -> None:
    d: dict[str, dict[str, list[float]]] = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(f"{prefix}_p*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f, newline="")):
            k = r["Kernel_Name"].split("(")[0]
            if k.startswith("void "):
                k = k[5:]
            d[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    med = {k: {c: statistics.median(v) for c, v in cs.items()} for k, cs in d.items()}

    def ratio(v, a, b, scale=1.0):
        return v[a] / (scale * v[b]) if v.get(a) is not None and v.get(b) else float("nan")
    rows = []
    for k, v in med.items():
        rows.append((k, ratio(v, "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_BUSY_CU_CYCLES", 4.0),
                     v.get("TCC_HIT_sum", 0.0) / max(1.0, v.get("TCC_HIT_sum", 0.0) + v.get("TCC_MISS_sum", 0.0)),
                     ratio(v, "SQ_WAIT_ANY", "SQ_WAVE_CYCLES"), ratio(v, "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE"),
                     ratio(v, "SQ_INSTS_VALU", "SQ_INSTS_MFMA")))
    rows.sort(key=lambda r: -(r[1] if r[1] == r[1] else -1))
    print(f"{'kernel':64s} {'mfma_busy':>9s} {'l2_hit':>7s} {'wait':>6s} {'lds_conf':>8s} {'VALU/MFMA':>10s}")
    for k, mb, l2, wt, lc, vm in rows:
        print(f"{k[:64]:64s} {mb:9.2f} {l2:7.2f} {wt:6.2f} {lc:8.3f} {vm:10.1f}")


if __name__ == "__main__":
    main(sys.argv[1])
