#!/usr/bin/env python3
"""Summarise tools/prof_traffic.sh output into profiles/:
  profiles/<tag>_kernel_stats.csv   rocprofv3 --stats summary (copied)
  profiles/<tag>_traffic.csv        per kernel: launches, avg ns, HBM bytes per launch
  profiles/traffic.json             {kernel: {hbm_bytes_per_step, launches_per_step}} for
                                    bench.py (the profiled run is one step, no warmup);
                                    profiles/traffic_configs4.json for --workload configs4-rank
HBM bytes = (r * FETCH_SIZE + WRITE_SIZE) * 1024 (counters in KiB).  r is the read
correction of the kernel's dominant read pattern, measured on known byte counts by
tools/calib_traffic.hip (profiles/calib_traffic.json): coalesced streaming reads are
reported at half their bytes (r = 2, as MI355X_MICROARCH.md documents), random 16-B loads
(k_probe's table probes) at 64 B each -- one 64-B request, r = 1.  WRITE_SIZE reads the
bytes of streaming stores exactly (calibrated 1.00) and counts a scattered 16-B store as
the 32 B it writes (2.00), so it is taken as is.  k_extend's own read patterns were
calibrated in round 3: its spill reloads (lane-interleaved 4-B words, k_lane_read4) report
0.50 of their bytes, like a coalesced stream, and its traceback's 2-B row-log reads
(k_log_read2) 0.88 -- a 128-B row read touching a second line half the time -- so r = 2
holds for k_extend too (profiles/calib_traffic.json).

    python tools/pmc_traffic.py <tag> [the bench.py arguments of the profiled run]

traffic.json's _method also records the workload key of the profiled run and the hash of
the HIP sources it ran (bench.source_hash): bench.py uses the figures only for a run of the
same workload on the same sources, and reports traffic: null otherwise.
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
PROF = os.path.join(ROOT, "profiles")
SHORT = {"k_extend": "k_extend", "k_probe": "k_probe", "k_probe_sorted": "k_probe_sorted",
         "k_chain": "k_chain",
         "k_fine": "k_fine", "k_table": "k_table", "k_coarse_scatter": "k_coarse_scatter",
         "k_coarse_hist": "k_coarse_hist", "k_pack": "k_pack"}


def short(name):
    for k in SHORT:
        if k + "(" in name or k + "<" in name:
            return k
    return None


def counters(tag, what, name=None):
    f = glob.glob(os.path.join(OUT, f"{tag}_{what}", "**", "*counter_collection.csv"),
                  recursive=True)
    tot, calls = defaultdict(float), defaultdict(set)
    for path in f:
        for row in csv.DictReader(open(path)):
            k = short(row["Kernel_Name"])
            if k and (name is None or row["Counter_Name"] == name):
                tot[k] += float(row["Counter_Value"])
                calls[k].add(row["Dispatch_Id"])
    return tot, {k: len(v) for k, v in calls.items()}


# read correction per kernel (see the docstring): k_probe's reads are random 16-B table
# entries; the others read mostly coalesced streams
READ_CORR = {"k_probe": 1.0}

N_SIMD = 1024          # 256 CUs x 4 SIMDs
VALU_ISSUE_CYC = 2     # MI355X_MICROARCH.md: a wave64 VALU instruction issues over 2 cycles


def issue(tag):
    """VALU issue fraction per kernel: SQ_INSTS_VALU x 2 cycles over the SIMD-cycles of its
    dispatches (GRBM_GUI_ACTIVE is summed over the 8 XCDs: cycles = GUI_ACTIVE / 8), and
    SALU instructions per CU-cycle."""
    valu, n = counters(tag, "issue", "SQ_INSTS_VALU")
    salu, _ = counters(tag, "issue", "SQ_INSTS_SALU")
    lds, _ = counters(tag, "issue", "SQ_INSTS_LDS")
    gui, _ = counters(tag, "issue", "GRBM_GUI_ACTIVE")
    out = {}
    for k in valu:
        cyc = gui.get(k, 0.0) / 8.0
        if cyc <= 0:
            continue
        out[k] = {"valu_insts": valu[k], "salu_insts": salu.get(k, 0.0),
                  "lds_insts": lds.get(k, 0.0), "gpu_cycles": cyc,
                  "valu_issue_frac": round(valu[k] * VALU_ISSUE_CYC / (N_SIMD * cyc), 4),
                  # one scalar unit per CU, shared by its 4 SIMDs: at most 1 SALU per cycle
                  "salu_per_cu_cycle": round(salu.get(k, 0.0) / (N_SIMD / 4 * cyc), 4)}
    return out


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
    os.makedirs(PROF, exist_ok=True)
    stats = glob.glob(os.path.join(OUT, f"{tag}_kt", "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        shutil.copy(stats[0], os.path.join(PROF, f"{tag}_kernel_stats.csv"))
    fetch, nf = counters(tag, "fetch")
    write, nw = counters(tag, "write")
    if not fetch or not write:
        sys.exit(f"no FETCH_SIZE / WRITE_SIZE passes for tag {tag} under {OUT}: "
                 "profiles/traffic.json left as it is")
    # instances of one kernel (k_extend's staged classes, k_probe<BLOOM>) add up: total time
    # over total calls
    tot_ns, calls_ns = defaultdict(float), defaultdict(int)
    if stats:
        for row in csv.DictReader(open(stats[0])):
            k = short(row["Name"])
            if k:
                tot_ns[k] += float(row["TotalDurationNs"])
                calls_ns[k] += int(row["Calls"])
    avg_ns = {k: tot_ns[k] / max(1, calls_ns[k]) for k in tot_ns}
    iss = issue(tag)
    traffic = {}
    with open(os.path.join(PROF, f"{tag}_traffic.csv"), "w") as f:
        f.write("kernel,launches,avg_ns,fetch_kib_per_launch,write_kib_per_launch,"
                "hbm_bytes_per_launch\n")
        for k in sorted(set(fetch) | set(write)):
            n = max(nf.get(k, 0), nw.get(k, 0), 1)
            fk, wk = fetch.get(k, 0.0) / n, write.get(k, 0.0) / n
            b = (READ_CORR.get(k, 2.0) * fk + wk) * 1024.0
            traffic[k] = {"hbm_bytes_per_step": int(b * n), "launches_per_step": n,
                          "hbm_bytes_per_launch": int(b)}
            if k in iss:
                traffic[k]["issue"] = iss[k]
            f.write(f"{k},{n},{avg_ns.get(k, 0):.0f},{fk:.1f},{wk:.1f},{b:.0f}\n")
    sys.path.insert(0, ROOT)
    import bench
    bargs = bench.parse_args(sys.argv[2:])
    jcls = bench.Configs4Rank if bargs.workload == "configs4-rank" else bench.Configs2
    traffic["_method"] = {"workload": jcls(bargs, 0, 1, None).workload_key(),
                          "src_sha": bench.source_hash(),
                          "hbm_bytes": "(r * FETCH_SIZE + WRITE_SIZE) KiB",
                          "read_correction": {"default": 2.0, **READ_CORR},
                          "calibration": "profiles/calib_traffic.json (tools/calib_traffic.hip)",
                          "tag": tag}
    with open(os.path.join(PROF, bench.TRAFFIC_FILES[bargs.workload]), "w") as f:
        json.dump(traffic, f, indent=1, sort_keys=True)
    print(json.dumps(traffic, indent=1))


if __name__ == "__main__":
    main()
