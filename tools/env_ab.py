#!/usr/bin/env python3
"""Interleaved A/B of environment knobs (read once per process by the
library, so every setting runs in its own process).

    python tools/env_ab.py --config e2e --rounds 3 --set "A:" --set "B:CIO_GPU_DMA_SUB_MB=0" \
        [--bench-args "--steps 30 --warmup 10 --no-cpu"] [--out gpurun_out/ab.jsonl]

Each round runs every setting once (`bench.py --config C ...` with the
setting's environment, a per-run time limit) and prints the line's value
plus the fields named by --fields (dotted paths into the bench JSON line).
"""
import argparse
import json
import os
os.environ.setdefault("CIO_GPU_DIAG", "1")   # the library honours its A/B switches only with this
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def dig(d, path):
    for k in path.split("."):
        if not isinstance(d, dict) or k not in d:
            return None
        d = d[k]
    return d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="e2e")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--set", action="append", required=True, help="NAME:VAR=val,VAR2=val")
    ap.add_argument("--bench-args", default="--steps 30 --warmup 10 --no-cpu")
    ap.add_argument("--fields", default="")
    ap.add_argument("--timeout", type=int, default=150)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    sets = []
    for s in args.set:
        name, _, kv = s.partition(":")
        env = dict(x.split("=", 1) for x in kv.split(",") if x)
        sets.append((name, env))
    fields = [f for f in args.fields.split(",") if f]
    res = {name: [] for name, _ in sets}
    out = open(args.out, "a") if args.out else None
    for r in range(args.rounds):
        for name, env in sets:
            e = dict(os.environ, **env)
            cmd = ["timeout", "-k", "10", str(args.timeout), sys.executable, os.path.join(ROOT, "bench.py"),
                   "--config", args.config] + args.bench_args.split()
            p = subprocess.run(cmd, env=e, capture_output=True, text=True)
            if p.returncode != 0:
                print(f"{name} round {r}: rc {p.returncode}\n{p.stderr[-2000:]}", flush=True)
                sys.exit(p.returncode)
            line = json.loads(p.stdout.strip().splitlines()[-1])
            row = {"set": name, "env": env, "round": r, "value": line.get("value")}
            for f in fields:
                row[f] = dig(line, f)
            res[name].append(row["value"])
            print(json.dumps(row), flush=True)
            if out:
                out.write(json.dumps(row) + "\n")
                out.flush()
    for name, vals in res.items():
        vals = [v for v in vals if v is not None]
        if vals:
            print(f"{name:>12}: mean {sum(vals) / len(vals):9.3f}  min {min(vals):9.3f}  max {max(vals):9.3f}  {vals}")


if __name__ == "__main__":
    main()
