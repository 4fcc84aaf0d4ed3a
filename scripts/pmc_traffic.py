"""Turn two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; separate runs, as
MI355X_MICROARCH.md §HBM prescribes) into profiles/pmc_traffic_<config>.json,
which bench.py reads as roofline.traffic when the schedule matches.

usage: python scripts/pmc_traffic.py CONFIG SCHEDULE PANEL_COLS KERNEL_SUBSTR FETCH_CSV WRITE_CSV [OUT]

FETCH_SIZE counts 1/2 of the bytes of 16-B/lane reads on gfx950 (the guide's
correction: bytes = 2 * FETCH_SIZE * 1024); WRITE_SIZE is exact for 16-B/lane
stores. Both are the L2 memory-side counters: Infinity-Cache hits are included."""

import csv
import json
import os
import sys


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
    cfg, schedule, panel_cols, kernel, fetch_csv, write_csv = sys.argv[1:7]
    out = sys.argv[7] if len(sys.argv) > 7 else os.path.join("profiles", f"pmc_traffic_{cfg}.json")
    fetch = per_launch(fetch_csv, kernel, "FETCH_SIZE")
    write = per_launch(write_csv, kernel, "WRITE_SIZE")
    fetch_b = 2.0 * 1024.0 * sum(fetch) / len(fetch)
    write_b = 1024.0 * sum(write) / len(write)
    rec = {
        "kernel": kernel,
        "config": cfg,
        "schedule": schedule,
        "panel_cols": int(panel_cols) if schedule != "tiled" else 0,
        "tiled_panel_cols": int(panel_cols) if schedule == "tiled" else None,
        "launches_per_spmm": 1,
        "source": [fetch_csv, write_csv],
        "FETCH_SIZE_KB_per_launch": fetch,
        "WRITE_SIZE_KB_per_launch": write,
        "correction": "gfx950 FETCH_SIZE counts 1/2 of the bytes of 16-B/lane reads (MI355X_MICROARCH.md §HBM): "
                      "fetch_bytes = 2 * FETCH_SIZE * 1024; WRITE_SIZE exact for 16-B/lane stores",
        "note": "L2 memory-side (fabric) traffic: Infinity Cache hits are included",
        "fetch_bytes": fetch_b,
        "write_bytes": write_b,
        "traffic_bytes_per_launch": fetch_b + write_b,
    }
    with open(out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps({k: rec[k] for k in ("kernel", "fetch_bytes", "write_bytes", "traffic_bytes_per_launch")}))


if __name__ == "__main__":
    main()
