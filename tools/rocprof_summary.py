"""Summarise rocprofv3 output for profiles/.

    python tools/rocprof_summary.py stats  <dir> <steps> [out.txt]
        per-kernel time per train step from <dir>/**/*kernel_stats.csv
    python tools/rocprof_summary.py shapes <dir> <steps> [top]
        per (kernel, grid) time per step from the kernel trace (which GEMM shape costs what)
    python tools/rocprof_summary.py kernel <dir> <kernel-substr> <grid> <min_us>
        average duration of the matching dispatches in <dir>/**/*kernel_trace.csv (cross-check
        of bench.py's live HIP-event timing of the roofline kernel)
    python tools/rocprof_summary.py traffic <fetch_dir> <write_dir> <kernel-substr> <grid> <min_us> [out.json]
        HBM bytes per launch of one kernel (dispatches matching name substring, grid size and
        a minimum duration, which separates GEMMs of the same tiling but different K)
        from two separate --pmc passes (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass).
    python tools/rocprof_summary.py pin [kind ...]
        copy the newest committed profiles/r*_<kind>_traffic.json (default: roofline, wgrad)
        into bench_pmc.json at the repository root, which bench.py reads on the GPU box
        (profiles/ is not shipped there).

Counter units and gfx950 corrections (MI355X_MICROARCH.md, HBM section; counter_defs.yaml):
FETCH_SIZE and WRITE_SIZE are kilobytes (expression / 1024); on gfx950 FETCH_SIZE reports
half the bytes of wide coalesced reads (16 B/lane global_load and buffer_load ... lds), so
bytes_read = 2 * 1024 * FETCH_SIZE; WRITE_SIZE is exact for 16 B/lane stores and fp32 atomics.
"""
import csv
import glob
import json
import os
import sys


def _find(d, suffix):
    hits = sorted(glob.glob(os.path.join(d, "**", "*" + suffix), recursive=True))
    if not hits:
        raise SystemExit(f"no *{suffix} under {d}")
    return hits


def stats(d, steps, out=None):
    rows = []
    for f in _find(d, "kernel_stats.csv"):
        rows += list(csv.DictReader(open(f)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    lines = [f"kernel time per step: {tot / steps / 1e6:.3f} ms  ({steps} steps profiled, "
             f"includes warm-up launches if the run had any)"]
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
        lines.append(f'{float(r["TotalDurationNs"]) / steps / 1e6:8.3f} ms/step '
                     f'{float(r["AverageNs"]) / 1e3:9.1f} us avg {int(r["Calls"]):6d} calls  '
                     f'{r["Name"][:110]}')
    txt = "\n".join(lines)
    if out:
        open(out, "w").write(txt + "\n")
    print(txt)


def shapes(d, steps, top=40):
    import collections
    g = collections.defaultdict(list)
    for f in _find(d, "kernel_trace.csv"):
        for r in csv.DictReader(open(f)):
            key = (r["Kernel_Name"][:70], r["Grid_Size_X"], r["Grid_Size_Z"], r["Workgroup_Size_X"])
            g[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for k, v in sorted(g.items(), key=lambda kv: -sum(kv[1]))[:top]:
        print(f"{sum(v) / steps / 1e3:7.3f} ms/step {len(v) / steps:5.1f}/step "
              f"avg {sum(v) / len(v):8.1f} us  grid {k[1]}x{k[2]} wg {k[3]}  {k[0]}")


def kernel(d, name_sub, grid, min_us):
    durs = []
    for f in _find(d, "kernel_trace.csv"):
        for r in csv.DictReader(open(f)):
            if name_sub not in r["Kernel_Name"] or int(r["Grid_Size_X"]) != grid:
                continue
            us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            if us >= min_us:
                durs.append(us)
    if not durs:
        raise SystemExit("no matching dispatches")
    print(f"{name_sub} grid {grid} (>= {min_us} us): {len(durs)} dispatches, "
          f"avg {sum(durs) / len(durs):.1f} us, min {min(durs):.1f}, max {max(durs):.1f}")


def gaps(d, marker="adamw_vec_kernel", last=10, out=None):
    """GPU-idle time per train step: steps are delimited by the end of the one AdamW launch per
    step (``marker``); within a step, idle = wall time - |union of every kernel's busy interval
    over all streams|.  Reported for the ``last`` steps of the trace (the timed region)."""
    ev = []
    for f in _find(d, "kernel_trace.csv"):
        for r in csv.DictReader(open(f)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                       r.get("Queue_Id", r.get("Stream_Id", ""))))
    ev.sort()
    ends = sorted(e for s, e, n, _ in ev if marker in n)
    if len(ends) < 2:
        raise SystemExit(f"fewer than 2 {marker} dispatches")
    rows = []
    for a, b in list(zip(ends[:-1], ends[1:]))[-last:]:
        iv = sorted((max(s, a), min(e, b)) for s, e, _, _ in ev if e > a and s < b)
        busy, cur_s, cur_e, n = 0, None, None, 0
        for s, e in iv:
            n += 1
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        if cur_e is not None:
            busy += cur_e - cur_s
        rows.append(((b - a) / 1e6, busy / 1e6, n))
    wall = sorted(r[0] for r in rows)[len(rows) // 2]
    idle = sorted(r[0] - r[1] for r in rows)[len(rows) // 2]
    res = {"steps": len(rows), "median_step_ms": wall, "median_gpu_idle_ms": idle,
           "median_busy_ms": sorted(r[1] for r in rows)[len(rows) // 2],
           "launches_per_step": rows[-1][2],
           "per_step": [{"wall_ms": w, "busy_ms": bz, "launches": n} for w, bz, n in rows]}
    if out:
        json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "per_step"}))


def _short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("((")[0].split("(float")[0].split("(bool")[0].split("(long")[0][:52]


def timeline(d, marker="embed_fwd_kernel", anchor="attn_bwd_dq_kernel<192, 1, 8>", layer=0,
             out=None):
    """Per-stream timeline of one decoder layer's backward in the last profiled step: every
    dispatch on every queue between the end of the (layer+1)-th-from-last ``anchor`` dispatch
    before it (or 1.6 ms earlier) and the first main-queue dispatch 300 us after this layer's
    anchor; plus the step's kernel time per queue.  Steps are delimited by ``marker``."""
    ev = []
    for f in _find(d, "kernel_trace.csv"):
        for r in csv.DictReader(open(f)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                       int(r["Queue_Id"]), int(r["Grid_Size_X"]), int(r["Grid_Size_Z"])))
    ev.sort()
    starts = [s for s, e, n, *_ in ev if marker in n]
    if len(starts) < 2:
        raise SystemExit(f"fewer than 2 {marker} dispatches")
    a, b = starts[-2], starts[-1]
    step = [x for x in ev if a <= x[0] < b]
    anchors = [x for x in step if anchor in x[2]]
    if not anchors:
        raise SystemExit(f"no {anchor} in the last step")
    # the backward walks the decoder from the last layer: anchors[0] is layer L-1
    k = anchors[layer]
    lo = anchors[layer - 1][1] if layer > 0 else k[0] - 1600_000
    hi = k[1] + 300_000
    lines = [f"# one decoder layer's backward (anchor {anchor} #{layer} of the last step), "
             f"us from the step start; q = HIP queue (one per stream)",
             f"# {'q':>2} {'start':>9} {'end':>9} {'us':>7}  kernel"]
    for s, e, n, q, gx, gz in step:
        if e <= lo or s >= hi:
            continue
        lines.append(f"  {q:2d} {(s - a) / 1e3:9.1f} {(e - a) / 1e3:9.1f} {(e - s) / 1e3:7.1f}  "
                     f"{_short(n):52s} grid {gx} z {gz}")
    per_q = {}
    for s, e, n, q, *_ in step:
        per_q[q] = per_q.get(q, 0) + (e - s)
    lines.append("")
    lines.append("# kernel time per queue in the step (us): " +
                 json.dumps({str(q): round(v / 1e3, 1) for q, v in sorted(per_q.items())}) +
                 f"  step wall {(b - a) / 1e3:.1f} us, {len(step)} launches")
    txt = "\n".join(lines)
    if out:
        open(out, "w").write(txt + "\n")
    print(txt)


def pmc(out, subs, *dirs):
    """Per (kernel, grid) averages of every counter collected in the --pmc pass directories
    ``dirs`` (one counter set per pass), for kernels whose name contains one of the
    comma-separated substrings ``subs``.  Counter values are summed over a dispatch's rows
    (per-XCD / per-SE instances), then averaged over dispatches; avg_us from the same rows."""
    import collections
    acc = collections.defaultdict(lambda: collections.defaultdict(dict))
    dur = collections.defaultdict(dict)
    want = [s for s in subs.split(",") if s]
    for d in dirs:
        for f in _find(d, "counter_collection.csv"):
            for r in csv.DictReader(open(f)):
                name = r["Kernel_Name"]
                if want and not any(w in name for w in want):
                    continue
                key = (name[:90], int(r["Grid_Size"]))
                disp = (f, r["Dispatch_Id"])
                c = acc[key][r["Counter_Name"]]
                c[disp] = c.get(disp, 0.0) + float(r["Counter_Value"])
                dur[key][disp] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    res = []
    for key, cs in acc.items():
        row = {"kernel": key[0], "grid": key[1],
               "avg_us": sum(dur[key].values()) / len(dur[key]), "dispatches": len(dur[key])}
        for cn, v in cs.items():
            row[cn] = sum(v.values()) / len(v)
        if "FETCH_SIZE" in row:
            row["hbm_read_bytes"] = 2.0 * 1024.0 * row["FETCH_SIZE"]
        if "WRITE_SIZE" in row:
            row["hbm_write_bytes"] = 1024.0 * row["WRITE_SIZE"]
        if "SQ_VALU_MFMA_BUSY_CYCLES" in row and "GRBM_GUI_ACTIVE" in row:
            # MFMA busy cycles summed over every SIMD of the chip (4 per CU x 256 CUs) vs the
            # kernel's GPU-active cycles (GRBM_GUI_ACTIVE is summed over the 8 XCDs)
            row["mfma_busy_frac"] = row["SQ_VALU_MFMA_BUSY_CYCLES"] / (
                1024.0 * row["GRBM_GUI_ACTIVE"] / 8.0)
        res.append(row)
    res.sort(key=lambda r: -r["avg_us"] * r["dispatches"])
    json.dump(res, open(out, "w"), indent=1)
    for r in res:
        print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.items()}))


def _per_dispatch(d, counter, name_sub, grid, min_us):
    vals = {}
    for f in _find(d, "counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter or name_sub not in r["Kernel_Name"]:
                continue
            if int(r["Grid_Size"]) != grid:
                continue
            if (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) < min_us * 1e3:
                continue
            key = (f, r["Dispatch_Id"])
            vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    if not vals:
        raise SystemExit(f"no {counter} rows for {name_sub!r} grid {grid} under {d}")
    return list(vals.values())


def traffic(fdir, wdir, name_sub, grid, min_us, out=None):
    fk = _per_dispatch(fdir, "FETCH_SIZE", name_sub, grid, min_us)
    wk = _per_dispatch(wdir, "WRITE_SIZE", name_sub, grid, min_us)
    rd = 2.0 * 1024.0 * sum(fk) / len(fk)
    wr = 1024.0 * sum(wk) / len(wk)
    res = {"kernel_substr": name_sub, "grid_size": grid, "min_us": min_us,
           "dispatches": [len(fk), len(wk)],
           "read_bytes_per_launch": rd, "write_bytes_per_launch": wr,
           "hbm_bytes_per_launch": rd + wr,
           "correction": "read = 2*1024*FETCH_SIZE (gfx950 half-count), write = 1024*WRITE_SIZE"}
    if out:
        json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


def pin(kinds=("roofline", "wgrad")):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = {}
    for kind in kinds:
        hits = sorted(glob.glob(os.path.join(root, "profiles", f"r*_{kind}_traffic.json")))
        if hits:
            d = json.load(open(hits[-1]))
            out[kind] = {"kernel_substr": d["kernel_substr"],
                         "hbm_bytes_per_launch": d["hbm_bytes_per_launch"],
                         "read_bytes_per_launch": d["read_bytes_per_launch"],
                         "write_bytes_per_launch": d["write_bytes_per_launch"],
                         "source": os.path.relpath(hits[-1], root)}
    json.dump(out, open(os.path.join(root, "bench_pmc.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "stats":
        stats(sys.argv[2], int(sys.argv[3]), sys.argv[4] if len(sys.argv) > 4 else None)
    elif sys.argv[1] == "shapes":
        shapes(sys.argv[2], int(sys.argv[3]), int(sys.argv[4]) if len(sys.argv) > 4 else 40)
    elif sys.argv[1] == "kernel":
        kernel(sys.argv[2], sys.argv[3], int(sys.argv[4]), float(sys.argv[5]))
    elif sys.argv[1] == "pmc":
        pmc(sys.argv[2], sys.argv[3], *sys.argv[4:])
    elif sys.argv[1] == "gaps":
        gaps(sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else "adamw_vec_kernel",
             int(sys.argv[4]) if len(sys.argv) > 4 else 10,
             sys.argv[5] if len(sys.argv) > 5 else None)
    elif sys.argv[1] == "timeline":
        timeline(sys.argv[2], layer=int(sys.argv[3]) if len(sys.argv) > 3 else 0,
                 out=sys.argv[4] if len(sys.argv) > 4 else None)
    elif sys.argv[1] == "traffic":
        traffic(sys.argv[2], sys.argv[3], sys.argv[4], int(sys.argv[5]), float(sys.argv[6]),
                sys.argv[7] if len(sys.argv) > 7 else None)
    elif sys.argv[1] == "pin":
        pin(tuple(sys.argv[2:]) or ("roofline", "wgrad"))
    else:
        raise SystemExit(__doc__)
