#!/usr/bin/env python3
"""Instruction mix of a kernel's hottest loop in a device assembly file
(hipcc --cuda-device-only -S): scripts/perf/isa_loop_stats.py FILE.s SYMBOL_SUBSTRING
Finds the function, then the loop whose back-edge branch spans the most
instructions, and counts waits, AGPR moves, memory and DPP instructions."""
import collections
import re
import sys


def main():
    path, sym = sys.argv[1], sys.argv[2]
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l) and sym in l)
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    body = lines[start:end]
    labels = {l.split(":")[0]: i for i, l in enumerate(body) if re.match(r"^\.LBB\S+:", l)}
    best = None
    for i, l in enumerate(body):
        m = re.match(r"\s+s_cbranch_\w+\s+(\.LBB\S+)", l) or re.match(r"\s+s_branch\s+(\.LBB\S+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            span = i - labels[m.group(1)]
            if best is None or span > best[1] - best[0]:
                best = (labels[m.group(1)], i)
    loop = [l.strip() for l in body[best[0]:best[1] + 1] if l.strip() and not l.strip().startswith(";")
            and not l.strip().startswith(".")]
    c = collections.Counter()
    waits = collections.Counter()
    for l in loop:
        op = l.split()[0]
        if op == "s_waitcnt":
            m = re.search(r"vmcnt\((\d+)\)", l)
            if m:
                waits[int(m.group(1))] += 1
            c["s_waitcnt"] += 1
        elif op.startswith("v_accvgpr"):
            c["v_accvgpr_*"] += 1
        elif op.startswith("global_load"):
            c[op] += 1
        elif op.startswith("ds_"):
            c[op] += 1
        elif "_dpp" in op or "dpp" in l:
            c["dpp"] += 1
        elif op.startswith("scratch") or op.startswith("buffer"):
            c["scratch/buffer"] += 1
        elif op.startswith("v_mov"):
            c["v_mov"] += 1
        elif op.startswith("v_add_f64") or op.startswith("v_mul_f64"):
            c[op] += 1
    meta = {}
    for l in lines[end:end + 60]:
        m = re.match(r"\s+\.(vgpr_count|agpr_count|sgpr_count|vgpr_spill_count|sgpr_spill_count):\s+(\d+)", l)
        if m:
            meta[m.group(1)] = int(m.group(2))
    for l in lines[start:end]:
        m = re.match(r"\s*;\s*(NumVgprs|NumAgprs|TotalNumVgprs|ScratchSize|Occupancy):\s*(\d+)", l)
        if m:
            meta[m.group(1)] = int(m.group(2))
    print(f"function: {body[0].split(':')[0]}")
    print(f"loop: {len(loop)} instructions")
    for k, v in sorted(c.items()):
        print(f"  {k}: {v}")
    print("  vmcnt waits (depth: count):", dict(sorted(waits.items())))
    print("  registers:", meta)


if __name__ == "__main__":
    main()
