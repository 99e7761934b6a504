"""Summarise the rocprofv3 outputs of tools/profile.sh (gpurun_out/prof_*) into one text table per kernel.

HBM bytes follow MI355X_MICROARCH.md's HBM section: FETCH_SIZE is in KB and reports half of the bytes of a wide
streaming read on gfx950 (so it is doubled here); WRITE_SIZE is taken as is. SQ_WAVE_CYCLES / SQ_WAIT_* /
SQ_ACTIVE_* count quad-cycles. Values are per launch (counter sum / launches of that kernel in the pass).

usage: python tools/summarize_prof.py gpurun_out [out.txt] [--traffic tools/pmc_traffic_c2.json --source NAME]
                                     [--workload '{"series": ..., "T": ..., "p": .., "d": .., "q": .., "I": .., "smear": ..,
                                                   "fit_kernel": 0, "options": ""}']
(--traffic adds k_cg_fit's measured HBM bytes per launch -- for a C5 workload ({"config": "c5", ...}) the whole
 order-search step's bytes -- keyed by the workload AND the sha256 of the profiled
 library spark-timeseries_amd/libsparkts_arima.so, to the record list bench.py reads for roofline.traffic; bench.py
 reports them only for the same workload and build. Default workload: bench.py's C2 run that tools/profile.sh profiles)
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def short(name):
    name = name.split("(")[0]
    return name.replace("void ", "").replace("sts::", "")


def kernel_stats(root):
    out = {}
    for f in glob.glob(os.path.join(root, "prof_trace", "*kernel_stats.csv")):
        for r in csv.DictReader(open(f)):
            out[short(r["Name"])] = (int(r["Calls"]), float(r["AverageNs"]))
    return out


def counters(root):
    acc = defaultdict(lambda: defaultdict(list))       # kernel -> counter -> [per-dispatch values]
    for f in glob.glob(os.path.join(root, "prof_*", "*counter_collection.csv")):
        per = defaultdict(float)
        meta = {}
        for r in csv.DictReader(open(f)):
            key = (r["Dispatch_Id"], short(r["Kernel_Name"]), r["Counter_Name"])
            per[key] += float(r["Counter_Value"])
            meta[r["Dispatch_Id"], short(r["Kernel_Name"])] = (r.get("VGPR_Count"), r.get("SGPR_Count"),
                                                               r.get("LDS_Block_Size"), r.get("Scratch_Size"))
        for (disp, k, c), v in per.items():
            acc[k][c].append(v)
        for (disp, k), m in meta.items():
            acc[k]["_meta"] = [m]
    return acc


def main():
    argv = list(sys.argv)
    traffic_path = source = None
    if "--traffic" in argv:
        i = argv.index("--traffic")
        traffic_path = argv[i + 1]
        del argv[i:i + 2]
    if "--source" in argv:
        i = argv.index("--source")
        source = argv[i + 1]
        del argv[i:i + 2]
    workload = {"series": 1048576, "T": 1024, "p": 2, "d": 1, "q": 2, "I": 1, "smear": 1, "fit_kernel": 0,
                "options": os.environ.get("SPARKTS_OPTIONS", "")}
    if "--workload" in argv:
        import json
        i = argv.index("--workload")
        workload = json.loads(argv[i + 1])
        del argv[i:i + 2]
    sys.argv = argv
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
    ks = kernel_stats(root)
    cs = counters(root)
    lines = []
    for k in sorted(set(ks) | set(cs), key=lambda x: -ks.get(x, (0, 0))[1]):
        calls, avg = ks.get(k, (0, 0.0))
        lines.append(f"== {k}: {calls} calls, avg {avg / 1e6:.3f} ms")
        c = cs.get(k, {})
        if "_meta" in c:
            v, s, l, sc = c["_meta"][0]
            lines.append(f"   VGPR {v}  SGPR {s}  LDS {l} B  scratch {sc} B")
        for name in sorted(x for x in c if x != "_meta"):
            vals = c[name]
            mean = sum(vals) / len(vals)
            extra = ""
            if name == "FETCH_SIZE":
                b = mean * 1024 * 2
                extra = f"  -> HBM read {b / 1e9:.3f} GB/launch (x2 gfx950 correction)"
                if avg:
                    extra += f", {b / (avg * 1e-9) / 1e9:.0f} GB/s at the traced avg duration"
            if name == "WRITE_SIZE":
                b = mean * 1024
                extra = f"  -> HBM write {b / 1e9:.3f} GB/launch"
            lines.append(f"   {name:28s} {mean:18.1f}{extra}")
    txt = "\n".join(lines)
    fit = next((v for k, v in cs.items() if k.startswith("k_cg_fit")), {})
    if traffic_path and workload.get("config") == "c5":
        # the order search: one step = every kernel of the 216 grid fits (all k_cg_fit / k_hr_init / k_ar_fit / ...
        # instantiations), so the record is the whole step's HBM bytes: the sum over every dispatch of the profiled
        # run (one step, no warmup) except the series sampler that fills the input
        import json
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                        "spark-timeseries_amd"))
        from sparkts_amd.buildinfo import library_sha, source_sha
        rd = sum(sum(c["FETCH_SIZE"]) for k, c in cs.items() if "sample" not in k and "FETCH_SIZE" in c) * 1024 * 2
        wr = sum(sum(c["WRITE_SIZE"]) for k, c in cs.items() if "sample" not in k and "WRITE_SIZE" in c) * 1024
        sha = library_sha()
        out = {"workload": workload, "build_sha": sha, "source_sha": source_sha(),
               "kernel": "every kernel of one order-search step", "hbm_bytes_per_step": rd + wr, "read_bytes": rd,
               "write_bytes": wr, "source": source or root}
        try:
            recs = json.load(open(traffic_path))
            recs = recs if isinstance(recs, list) else [recs]
        except (OSError, ValueError):
            recs = []
        recs = [r for r in recs if not (r.get("workload") == workload and r.get("build_sha") == sha)
                and r.get("build_sha")] + [out]
        json.dump(recs, open(traffic_path, "w"), indent=1)
        fit = {}
    if traffic_path and "FETCH_SIZE" in fit and "WRITE_SIZE" in fit:
        import json
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                        "spark-timeseries_amd"))
        from sparkts_amd.buildinfo import library_sha, source_sha
        rd = sum(fit["FETCH_SIZE"]) / len(fit["FETCH_SIZE"]) * 1024 * 2
        wr = sum(fit["WRITE_SIZE"]) / len(fit["WRITE_SIZE"]) * 1024
        sha = library_sha()
        out = {"workload": workload, "build_sha": sha, "source_sha": source_sha(),
               "kernel": "k_cg_fit", "hbm_bytes_per_launch": rd + wr, "read_bytes": rd, "write_bytes": wr,
               "source": source or root}

        def mean(name):
            return sum(fit[name]) / len(fit[name]) if name in fit else None
        wc = mean("SQ_WAVE_CYCLES")
        if wc:
            # quad-cycle counters summed over waves; one wave per SIMD, so these are fractions of SIMD time
            if mean("SQ_ACTIVE_INST_VALU") is not None:
                out["valu_busy"] = mean("SQ_ACTIVE_INST_VALU") / wc
            if mean("SQ_WAIT_ANY") is not None:
                out["wait_frac"] = mean("SQ_WAIT_ANY") / wc
        try:
            recs = json.load(open(traffic_path))
            recs = recs if isinstance(recs, list) else [recs]
        except (OSError, ValueError):
            recs = []
        recs = [r for r in recs if not (r.get("workload") == workload and r.get("build_sha") == sha)
                and r.get("build_sha")] + [out]
        json.dump(recs, open(traffic_path, "w"), indent=1)
    print(txt)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(txt + "\n")


if __name__ == "__main__":
    main()
