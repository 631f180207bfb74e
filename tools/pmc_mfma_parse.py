"""MFMA utilisation per kernel from tools/pmc_mfma.sh's pass -> profiles/pmc_mfma_c2.json.

MfmaUtil = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE x SIMDs) (rocprofv3's derived formula,
256 CUs x 4 SIMDs) with GRBM_GUI_ACTIVE divided by the 8 XCDs: on gfx950 the per-dispatch value
comes summed over the XCDs (the raw formula gives 1/8 of the flop-based fraction on every kernel);
MFMA flops = SQ_INSTS_VALU_MFMA_MOPS_F32 x 512 (the derived MfmaFlopsF32), achieved TF/s = flops /
kernel duration (same run's kernel trace) -- the two fractions agree within a few %."""
import csv
import glob
import json
import sys
from collections import defaultdict
from pathlib import Path

SIMDS = 256 * 4
XCDS = 8
PEAK_F32_TF = 157.3


def main():
    src, dst = Path(sys.argv[1]), Path(sys.argv[2])
    # one record per (run, kernel): a run is the first directory under src (several programs profiled
    # into one src keep their kernels apart, e.g. the same TransR kernel at two batch sizes)
    def tag(f):
        rel = Path(f).relative_to(src).parts
        return rel[0] if len(rel) >= 2 else ""

    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(str(src / "**" / "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            vals[(tag(f), row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
    dur = defaultdict(list)
    for f in glob.glob(str(src / "**" / "*kernel_trace.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            dur[(tag(f), row["Kernel_Name"])].append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    what = sys.argv[3] if len(sys.argv) > 3 else "tools/bench_kernels.py --only graph,attention,nfm (C2 shapes)"
    out = {"source": "rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 GRBM_GUI_ACTIVE "
                     "--kernel-trace -- " + what,
           "peak_f32_mfma_tflops": PEAK_F32_TF, "kernels": {}}
    for key, c in vals.items():
        run, name = key
        busy, mops, gui = (c.get(k, []) for k in ("SQ_VALU_MFMA_BUSY_CYCLES", "SQ_INSTS_VALU_MFMA_MOPS_F32",
                                                  "GRBM_GUI_ACTIVE"))
        if not busy or not gui or sum(mops) == 0:
            continue
        n = len(busy)
        rec = {"launches": n, "mfma_util": sum(busy) / n / (max(gui) / XCDS * SIMDS),
               "mfma_flops_per_launch": 512.0 * sum(mops) / len(mops)}
        d = dur.get(key)
        if d:
            rec["avg_us"] = sum(d) / len(d) / 1e3
            rec["achieved_tflops"] = rec["mfma_flops_per_launch"] / (rec["avg_us"] * 1e-6) / 1e12
            rec["frac_of_peak"] = rec["achieved_tflops"] / PEAK_F32_TF
        out["kernels"][(f"[{run}] " if run else "") + name[:120]] = rec
    dst.write_text(json.dumps(out, indent=1))
    for k, r in out["kernels"].items():
        print(f"{r.get('avg_us', 0):9.1f} us  util {r['mfma_util']:.3f}  {r.get('achieved_tflops', 0):6.1f} TF  {k[:80]}")


if __name__ == "__main__":
    main()
