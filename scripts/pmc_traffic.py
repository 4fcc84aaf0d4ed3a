"""Turn rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; separate runs, as
MI355X_MICROARCH.md §HBM prescribes) into profiles/pmc_traffic_<config>.json,
which bench.py reads as roofline.traffic when the schedule matches.

usage: python scripts/pmc_traffic.py CONFIG SCHEDULE PANEL_COLS KERNEL_SUBSTR FETCH_CSV WRITE_CSV
           [--probe FETCH_PROBE_CSV --stream-bytes B] [--out OUT]

The guide (MI355X_MICROARCH.md:298) calibrates FETCH_SIZE for 16-B/lane reads
only: it reports 1/2 of their bytes. The kernels also read their index /
value stream with 4-B and 8-B lanes, which the guide leaves uncalibrated. So
the stream is calibrated here on the kernel itself:

* --probe: a FETCH_SIZE pass of the same run with the kernel's probe mask at
  0 (BSM_TILED_PROBE_MASK, BSM_TILED_K1_PROBE or BSM_SPMM_PROBE_MASK), where
  every gather reads X row 0 (an L2 hit), so the counter sees the stream
  alone (wrong results: measurement only);
* --stream-bytes: the stream's true size (the tiled copy's bytes; it has no
  reuse, so every byte goes to memory once).

stream_factor = stream-bytes / (probe FETCH_SIZE x 1024), and
gather bytes = 2 x (FETCH_SIZE - probe FETCH_SIZE) x 1024 (16-B/lane, the
guide's 1/2). Traffic = stream-bytes + gather bytes + WRITE_SIZE x 1024
(exact for 16-B/lane stores). Without a probe the guide's 2x is applied to
all of FETCH_SIZE, which the C4 calibration supports (stream_factor 2.0).
Both counters are the L2's memory-side (fabric) counters: Infinity-Cache hits
are included."""

import argparse
import csv
import json
import os


def per_launch(path, kernel, counter):
    vals = []
    with open(path) as f:
        for row in csv.DictReader(f):
            if kernel in row["Kernel_Name"] and row["Counter_Name"] == counter:
                vals.append(float(row["Counter_Value"]))
    if not vals:
        raise SystemExit(f"{path}: no {counter} rows for a kernel matching {kernel!r}")
    return vals


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config")
    ap.add_argument("schedule")
    ap.add_argument("panel_cols", type=int)
    ap.add_argument("kernel")
    ap.add_argument("fetch_csv")
    ap.add_argument("write_csv")
    ap.add_argument("--probe", default=None)
    ap.add_argument("--probe-kernel", default=None, help="kernel name substring in the probe csv (default: kernel)")
    ap.add_argument("--stream-bytes", type=float, default=None)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    out = a.out or os.path.join("profiles", f"pmc_traffic_{a.config}.json")
    fetch = per_launch(a.fetch_csv, a.kernel, "FETCH_SIZE")
    write = per_launch(a.write_csv, a.kernel, "WRITE_SIZE")
    fetch_kb = sum(fetch) / len(fetch)
    write_b = 1024.0 * sum(write) / len(write)
    rec = {
        "kernel": a.kernel,
        "config": a.config,
        "schedule": a.schedule,
        "panel_cols": a.panel_cols if a.schedule != "tiled" else 0,
        "tiled_panel_cols": a.panel_cols if a.schedule == "tiled" else None,
        "launches_per_spmm": 1,
        "source": [a.fetch_csv, a.write_csv] + ([a.probe] if a.probe else []),
        "FETCH_SIZE_KB_per_launch": fetch,
        "WRITE_SIZE_KB_per_launch": write,
        "note": "L2 memory-side (fabric) traffic: Infinity Cache hits are included",
        "write_bytes": write_b,
    }
    if a.probe:
        probe = per_launch(a.probe, a.probe_kernel or a.kernel, "FETCH_SIZE")
        probe_kb = sum(probe) / len(probe)
        gather_b = 2.0 * 1024.0 * (fetch_kb - probe_kb)
        rec.update({
            "probe_FETCH_SIZE_KB_per_launch": probe,
            "stream_bytes": a.stream_bytes,
            "stream_factor": round(a.stream_bytes / (probe_kb * 1024.0), 4),
            "gather_bytes": gather_b,
            "correction": "stream calibrated on the kernel (a probe pass with every gather on X row 0: "
                          "BSM_TILED_PROBE_MASK=0 (k = 32 copy), BSM_TILED_K1_PROBE=0 (k = 1 copy), "
                          "BSM_SPMM_PROBE_MASK=0 (row kernel); the stream alone; stream_factor = true stream bytes "
                          "/ (probe FETCH_SIZE x 1024)); gathers: 2 x (FETCH_SIZE - probe) x 1024 "
                          "(MI355X_MICROARCH.md:298 for 16-B lanes; the 8-B lanes of k = 1 by the stream's own "
                          "factor, ~1.9); WRITE_SIZE exact",
            "fetch_bytes": a.stream_bytes + gather_b,
        })
    else:
        rec.update({
            "correction": "2 x FETCH_SIZE x 1024 for all reads (the guide's 16-B/lane 1/2, and the C4 stream "
                          "calibration: 4-B/8-B lanes also count 1/2, pmc_traffic_c4.json stream_factor)",
            "fetch_bytes": 2.0 * 1024.0 * fetch_kb,
        })
    rec["traffic_bytes_per_launch"] = rec["fetch_bytes"] + write_b
    with open(out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps({k: rec.get(k) for k in ("kernel", "stream_factor", "gather_bytes", "fetch_bytes", "write_bytes",
                                              "traffic_bytes_per_launch")}))


if __name__ == "__main__":
    main()
