"""Parse the two rocprofv3 --pmc passes of tools/pmc_bench.sh / pmc_spmm.sh into profiles/pmc_<cfg>.json.

gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports half
the bytes of a wide (16 B/lane) coalesced read -- the SpMM's row gathers are
16 B/lane float4 loads -- so it is doubled; WRITE_SIZE is exact for 16-B
stores.  Both counters are in KiB.  Averaged per launch of the forward SpMM
kernel (spmm_main_kernel<64, 0>) plus its fix-up (spmm_fixup_kernel<64, 0>).
"""
import csv
import glob
import json
import sys
from collections import defaultdict
from pathlib import Path


def per_kernel(path_glob, counter):
    vals = defaultdict(list)
    for f in glob.glob(path_glob, recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                vals[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return vals


def main():
    src, dst = Path(sys.argv[1]), Path(sys.argv[2])
    cmd = sys.argv[3] if len(sys.argv) > 3 else "tools/bench_kernels.py --only spmm"
    fetch = per_kernel(str(src / "FETCH_SIZE" / "**" / "*counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel(str(src / "WRITE_SIZE" / "**" / "*counter_collection.csv"), "WRITE_SIZE")
    out = {"source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), {cmd}",
           "correction": "FETCH_SIZE x2 (gfx950 wide-read undercount), KiB -> bytes", "kernels": {}}
    main_k = fix_k = tu_k = tu_fix = None
    d0 = int(sys.argv[4]) if len(sys.argv) > 4 else 64  # the forward SpMM's width (the bench's embed_dim)
    for name in set(fetch) | set(write):
        f = fetch.get(name, [])
        w = write.get(name, [])
        if not f or not w:
            continue
        rec = {"launches": len(f), "fetch_bytes": 2 * 1024 * sum(f) / len(f), "write_bytes": 1024 * sum(w) / len(w)}
        rec["hbm_bytes"] = rec["fetch_bytes"] + rec["write_bytes"]
        out["kernels"][name] = rec
        if f"spmm_main_kernel<{d0}, 0>" in name:
            main_k = rec
        if f"spmm_fixup_kernel<{d0}, 0>" in name:
            fix_k = rec
        if f"spmm_main_kernel<{d0}, 4>" in name:  # the layer-0 A^T product fused with the table's Adam
            tu_k = rec
        if f"spmm_fixup_kernel<{d0}, 4>" in name:
            tu_fix = rec
    if main_k:
        out["spmm_fwd_hbm_bytes_per_launch"] = main_k["hbm_bytes"] + (fix_k["hbm_bytes"] if fix_k else 0.0)
    if tu_k:
        out["table_update_hbm_bytes_per_launch"] = tu_k["hbm_bytes"] + (tu_fix["hbm_bytes"] if tu_fix else 0.0)
    if len(sys.argv) > 5:  # the bench log of the profiled run: the graph size the counters belong to
        import re
        text = Path(sys.argv[5]).read_text()
        # a rank share (bench.py --rank-share) files its counters under its own rows / entries of A
        m = re.search(r"share graph: N=(\d+) nnz=(\d+)", text) or re.search(r"graph: N=(\d+) .*nnz=(\d+)", text)
        if m:
            out["nodes"], out["nnz"] = int(m.group(1)), int(m.group(2))
    dst.write_text(json.dumps(out, indent=1))
    print(json.dumps(out.get("spmm_fwd_hbm_bytes_per_launch")))


if __name__ == "__main__":
    main()
