#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs: per-dispatch median/mean of each counter for one kernel.

    python tools/pmc_summary.py <dir> [kernel] [--json out.json]

With --json, also writes the per-launch HBM traffic of the kernel as MI355X_MICROARCH.md's
HBM/rocprofv3 section prescribes: FETCH_SIZE (kB) doubled (gfx950 reports half of the bytes of
wide coalesced reads) + WRITE_SIZE (kB), medians over the dispatches.
"""
import collections
import csv
import glob
import sys

args = [a for a in sys.argv[1:]]
jout = None
if "--json" in args:
    i = args.index("--json")
    jout = args[i + 1]
    del args[i:i + 2]
d = args[0]
kern = args[1] if len(args) > 1 else "k_env_step"
agg = collections.defaultdict(list)
for f in sorted(glob.glob(f"{d}/*counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if kern in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    v = sorted(v)
    print(f"{k:28s} n={len(v):3d} median={v[len(v)//2]:.4g} mean={sum(v)/len(v):.4g}")
if jout:
    import json
    med = {k: sorted(v)[len(v) // 2] for k, v in agg.items()}
    fetch, write = med.get("FETCH_SIZE"), med.get("WRITE_SIZE")
    out = {"kernel": kern, "dispatches": len(agg.get("FETCH_SIZE", [])), "FETCH_SIZE_kB": fetch, "WRITE_SIZE_kB": write,
           "traffic_bytes_per_launch": None if fetch is None or write is None else (2.0 * fetch + write) * 1024.0,
           "correction": "FETCH_SIZE x2 (gfx950, MI355X_MICROARCH.md HBM/rocprofv3); kB = 1024 B"}
    # issue / latency picture of the same launches (per-wave cycle fractions, medians over dispatches)
    wc = med.get("SQ_WAVE_CYCLES")
    if wc:
        out["issue"] = {k: med[c] / wc for k, c in (("valu_active_frac", "SQ_ACTIVE_INST_VALU"),
                                                     ("any_active_frac", "SQ_ACTIVE_INST_ANY"),
                                                     ("wait_any_frac", "SQ_WAIT_ANY"),
                                                     ("wait_inst_lds_frac", "SQ_WAIT_INST_LDS")) if c in med}
        if "SQ_INSTS_VALU" in med:
            out["issue"]["valu_insts_per_launch"] = med["SQ_INSTS_VALU"]
        if "SQ_INSTS_LDS" in med and "SQ_LDS_BANK_CONFLICT" in med:
            out["issue"]["lds_bank_conflict_cycles_per_lds_inst"] = med["SQ_LDS_BANK_CONFLICT"] / med["SQ_INSTS_LDS"]
    json.dump(out, open(jout, "w"), indent=1)
    print("wrote", jout)
