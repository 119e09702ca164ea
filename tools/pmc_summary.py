#!/usr/bin/env python3
"""Per-kernel table of the rocprofv3 PMC passes written by tools/pmc.sh.

  python tools/pmc_summary.py gpurun_out/pmc

For every dmlc:: kernel: dispatches, mean duration, and per dispatch the mean of each counter, plus
derived columns: MFMA busy share (SQ_VALU_MFMA_BUSY_CYCLES over GRBM_GUI_ACTIVE x 4 SIMDs x 256 CUs / 8
XCDs -- GRBM_GUI_ACTIVE sums the 8 XCDs), LDS bank-conflict share (SQ_LDS_BANK_CONFLICT /
SQ_LDS_IDX_ACTIVE), and HBM-side bytes (FETCH_SIZE is in KB and on gfx950 reports half the bytes of wide
streaming reads: MI355X_MICROARCH.md, so both the raw and the doubled figure are shown).
"""
import collections
import csv
import glob
import os
import sys


def load(pass_dir):
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(pass_dir, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                name = r["Kernel_Name"]
                if "dmlc::" not in name:
                    continue
                k = name.split("(")[0].replace("dmlc::", "").replace("void ", "")
                key = (k, r.get("Dispatch_Id") or r.get("Correlation_Id"))
                out[k][r["Counter_Name"]].append((key, float(r["Counter_Value"])))
    return out


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
    merged = collections.defaultdict(dict)
    for p in sorted(glob.glob(os.path.join(root, "*"))):
        if not os.path.isdir(p):
            continue
        for k, ctrs in load(p).items():
            for c, vals in ctrs.items():
                per = collections.defaultdict(float)       # sum over XCD / SE instances per dispatch
                for key, v in vals:
                    per[key] += v
                merged[k][c] = (sum(per.values()) / max(1, len(per)), len(per))
    cols = ["SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_LDS_IDX_ACTIVE",
            "SQ_LDS_BANK_CONFLICT", "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE", "FETCH_SIZE", "WRITE_SIZE"]
    extra = sorted({c for m in merged.values() for c in m} - set(cols))
    cols = [c for c in cols if any(c in m for m in merged.values())] + extra
    print("per dispatch means (counters summed over all instances of one dispatch)")
    hdr = ["kernel", "n"] + cols + ["mfma_busy%", "lds_conflict%", "fetch_MB(x2)", "write_MB"]
    print(" | ".join(hdr))
    for k in sorted(merged):
        m = merged[k]
        n = max(v[1] for v in m.values())
        row = [k, str(n)] + [f"{m[c][0]:.4g}" if c in m else "-" for c in cols]
        mf = m.get("SQ_VALU_MFMA_BUSY_CYCLES", (None,))[0]
        gui = m.get("GRBM_GUI_ACTIVE", (None,))[0]
        busy = f"{100.0 * mf / (gui / 8 * 4 * 256):.1f}" if mf is not None and gui else "-"
        lds = m.get("SQ_LDS_IDX_ACTIVE", (None,))[0]
        cf = m.get("SQ_LDS_BANK_CONFLICT", (None,))[0]
        conf = f"{100.0 * cf / lds:.1f}" if lds and cf is not None else "-"
        fe = m.get("FETCH_SIZE", (None,))[0]
        wr = m.get("WRITE_SIZE", (None,))[0]
        row += [busy, conf, f"{fe / 1024:.2f} ({2 * fe / 1024:.2f})" if fe is not None else "-",
                f"{wr / 1024:.2f}" if wr is not None else "-"]
        print(" | ".join(row))


if __name__ == "__main__":
    main()
