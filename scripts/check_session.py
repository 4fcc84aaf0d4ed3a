#!/usr/bin/env python3
"""Validate a GPU session file before spending GPU minutes: every
"py:<script> <args>" / "pmc:<config>:<counters>:<extra>" / "bench:..." step's
arguments must parse with that script's own argparse (parsing only: the
script stops right after parse_args), and every "tests:<paths>" path must
exist. Usage: python scripts/check_session.py scripts/sess_XXX.sh"""
import argparse
import os
import re
import runpy
import shlex
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def check_args(script, args):
    code = ("import argparse, runpy, sys\n"
            "orig = argparse.ArgumentParser.parse_args\n"
            "def pa(self, *a, **k):\n"
            "    orig(self, *a, **k)\n"
            "    sys.exit(0)\n"
            "argparse.ArgumentParser.parse_args = pa\n"
            f"sys.argv = {[script] + args!r}\n"
            f"runpy.run_path({script!r}, run_name='__main__')\n")
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=300)
    return r.returncode == 0, (r.stderr or r.stdout)[-400:]


def main():
    text = open(sys.argv[1]).read()
    # shell variables defined in the file (simple NAME="..." lines)
    env = dict(re.findall(r'^([A-Z_]+)="([^"]*)"', text, re.M))
    steps = re.findall(r'"((?:py|tests|pmc|bench|prof):[^"]*)"', text)
    ok_all = True
    for st in steps:
        st = re.sub(r"\$(\w+)", lambda m: env.get(m.group(1), m.group(0)), st)
        kind, _, rest = st.partition(":")
        if kind == "py":
            parts = shlex.split(rest)
            ok, msg = check_args(parts[0], parts[1:])
        elif kind in ("pmc", "bench", "prof"):
            fields = rest.split(":")
            cfg = fields[0]
            extra = fields[-1] if (kind == "pmc" and len(fields) > 2) or (kind != "pmc" and len(fields) > 1) else ""
            ok, msg = check_args("bench.py", ["--config", cfg] + shlex.split(extra))
        else:
            paths = [p.split("::")[0] for p in shlex.split(rest)]
            missing = [p for p in paths if not os.path.exists(os.path.join(ROOT, p))]
            ok, msg = not missing, f"missing {missing}"
        print(("ok   " if ok else "FAIL ") + st[:120] + ("" if ok else "\n     " + msg.strip().replace("\n", "\n     ")))
        ok_all &= ok
    sys.exit(0 if ok_all else 1)


if __name__ == "__main__":
    main()
