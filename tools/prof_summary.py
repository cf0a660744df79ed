"""Fold one round's rocprofv3 outputs (tools/profile_round.sh) into profiles/.

  python tools/prof_summary.py gpurun_out/r01 --tag r01 --out profiles

Reads  <dir>/trace/run_kernel_stats.csv           (--kernel-trace --stats)
       <dir>/pmc_fetch/run_counter_collection.csv  (--pmc FETCH_SIZE)
       <dir>/pmc_write/run_counter_collection.csv  (--pmc WRITE_SIZE)
       <dir>/bench_trace.json                      (the bench line of the traced run)
Writes <out>/<tag>_kernel_stats.csv, <out>/<tag>_summary.md, <out>/<tag>_traffic.json.

HBM bytes per launch (MI355X_MICROARCH.md, HBM/rocprofv3 section): FETCH_SIZE
and WRITE_SIZE are KiB; on gfx950 FETCH_SIZE reports half the bytes of a
coalesced streaming read, so fetched bytes = 2 x FETCH_SIZE x 1024.  The
correction is calibrated in our own access pattern by k_radix_hist, which reads
exactly 4 B per message (the group ids) and writes a 64-bin histogram per tile.
"""
import argparse
import csv
import json
import os
import shutil
from collections import defaultdict


def short(name):
    return name.split("(")[0].replace("void ", "")


def kernel_stats(path):
    rows = {}
    for r in csv.DictReader(open(path)):
        rows[short(r["Name"])] = {"calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3,
                                  "min_us": float(r["MinNs"]) / 1e3, "max_us": float(r["MaxNs"]) / 1e3,
                                  "total_pct": float(r["Percentage"])}
    return rows


def counter(path, name):
    acc = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == name:
            acc[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return acc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--tag", default="r01")
    ap.add_argument("--out", default="profiles")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    ks_path = os.path.join(a.dir, "trace", "run_kernel_stats.csv")
    ks = kernel_stats(ks_path)
    shutil.copy(ks_path, os.path.join(a.out, f"{a.tag}_kernel_stats.csv"))
    fetch = counter(os.path.join(a.dir, "pmc_fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = counter(os.path.join(a.dir, "pmc_write", "run_counter_collection.csv"), "WRITE_SIZE")
    bench = None
    bpath = os.path.join(a.dir, "bench_trace.json")
    if os.path.exists(bpath):
        lines = [ln for ln in open(bpath) if ln.startswith("{")]
        bench = json.loads(lines[-1]) if lines else None
    nmsg = bench["config"].get("msgappresp_per_step") if bench else None

    def traffic(k):
        f = fetch.get(k)
        w = write.get(k)
        if not f or not w:
            return None
        # skip the first (cold) launches of the warmup; average the rest
        f = f[2:] or f
        w = w[2:] or w
        fb = 2.0 * 1024.0 * sum(f) / len(f)
        wb = 1024.0 * sum(w) / len(w)
        return {"fetch_kib_raw": sum(f) / len(f), "fetch_bytes": fb, "write_bytes": wb, "traffic_bytes": fb + wb,
                "launches": len(f)}

    out = {"tag": a.tag, "kernels": {}}
    lines = [f"# {a.tag}: rocprofv3 kernel trace + HBM traffic (MI355X, 1 GPU)", ""]
    if bench:
        lines += [f"bench (traced run): value {bench['value']:.4g} {bench['unit']}, "
                  f"ms_per_step {bench['ms_per_step']:.4f}, phases {json.dumps(bench.get('phases'))}", ""]
    lines += ["| kernel | calls | avg µs | min µs | % time | fetch B/launch (2×FETCH_SIZE) | write B/launch | "
              "traffic B/launch | GB/s at avg |", "|---|---|---|---|---|---|---|---|---|"]
    for k, s in sorted(ks.items(), key=lambda kv: -kv[1]["total_pct"]):
        t = traffic(k)
        out["kernels"][k] = dict(s, **(t or {}))
        if t:
            gbs = t["traffic_bytes"] / (s["avg_us"] * 1e-6) / 1e9
            lines.append(f"| {k} | {s['calls']} | {s['avg_us']:.1f} | {s['min_us']:.1f} | {s['total_pct']:.1f} | "
                         f"{t['fetch_bytes']:.4g} | {t['write_bytes']:.4g} | {t['traffic_bytes']:.4g} | {gbs:.0f} |")
        else:
            lines.append(f"| {k} | {s['calls']} | {s['avg_us']:.1f} | {s['min_us']:.1f} | {s['total_pct']:.1f} "
                         f"| - | - | - | - |")
    cal = traffic("k_radix_hist")
    if cal and nmsg:
        exp = 4.0 * nmsg
        lines += ["", f"Calibration: k_radix_hist reads exactly 4 B x {nmsg} messages = {exp:.4g} B; "
                      f"2 x FETCH_SIZE = {cal['fetch_bytes']:.4g} B (ratio {cal['fetch_bytes'] / exp:.3f})."]
        out["calibration"] = {"kernel": "k_radix_hist", "expected_read_bytes": exp,
                              "measured_read_bytes": cal["fetch_bytes"]}
    # the whole step (every kernel hb_step launches, per step; k_route runs once per step)
    step_k = ("k_radix_hist", "k_scan_rows", "k_radix_scatter", "k_bucket_bounds", "k_route", "k_apply", "k_elect",
              "k_follow", "k_finish", "k_tick")
    steps = sum(s["calls"] for k, s in ks.items() if k.startswith("k_route"))
    if not steps:  # a Tick line (hb_tick: k_tick + k_finish per tick)
        steps = sum(s["calls"] for k, s in ks.items() if k.startswith("k_tick<"))
    if steps:
        tb = us = 0.0
        missing = []
        for k, s in ks.items():
            if not k.startswith(step_k):
                continue
            us += s["avg_us"] * s["calls"] / steps
            t = traffic(k)
            if t:
                tb += t["traffic_bytes"] * s["calls"] / steps
            else:
                missing.append(k)
        out["step"] = {"traffic_bytes": tb, "kernel_us": us, "steps": steps, "kernels_without_pmc": missing}
        lines += ["", f"Whole step ({steps} steps traced): kernels {us:.1f} us, HBM traffic {tb:.4g} B per step "
                      f"(FETCH_SIZE x 2 + WRITE_SIZE summed over the step's kernels)"]
    if bench:
        out["bench"] = {"value": bench["value"], "ms_per_step": bench["ms_per_step"], "phases": bench.get("phases"),
                        "config": bench["config"]}
    open(os.path.join(a.out, f"{a.tag}_summary.md"), "w").write("\n".join(lines) + "\n")
    json.dump(out, open(os.path.join(a.out, f"{a.tag}_traffic.json"), "w"), indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
