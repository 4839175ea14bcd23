"""Summarise a rocprofv3 kernel trace over the last N training steps.

    python scripts/prof_summary.py <kernel_trace.csv> --steps 10 --per-step-marker sgd_flat_kernel \
        --markers-per-step 5 [--title ...] > profiles/xxx.md

Step boundaries are found from a kernel that runs a fixed number of times per
step (the fused optimizer kernel: one launch per gradient bucket).  Prints a
markdown table: ms/step, % of GPU-busy time, launches/step per kernel, plus the
GPU-busy and wall span per step (overlapping kernels on the comm stream count
once in the span, twice in busy).
"""
import argparse
import csv
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--per-step-marker", default="sgd_flat_kernel")
    ap.add_argument("--markers-per-step", type=int, default=5)
    ap.add_argument("--total-steps", type=int, default=0,
                    help="steps the profiled run executed in all (infers markers per step)")
    ap.add_argument("--title", default="")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    marks = [i for i, r in enumerate(rows) if a.per_step_marker in r[2]]
    if a.total_steps:
        a.markers_per_step = len(marks) // a.total_steps
    need = a.markers_per_step * (a.steps + 1)
    if len(marks) < need:
        raise SystemExit(f"only {len(marks)} marker launches, need {need}")
    start_i = marks[-need + a.markers_per_step - 1] + 1   # after the last marker of step -(N+1)
    end_i = marks[-1] + 1
    win = rows[start_i:end_i]
    tot = defaultdict(float)
    cnt = defaultdict(int)
    for s, e, n in win:
        tot[n] += (e - s) / 1e6
        cnt[n] += 1
    busy = sum(tot.values())
    span = (win[-1][1] - win[0][0]) / 1e6
    if a.title:
        print(f"# {a.title}\n")
    print(f"GPU busy {busy / a.steps:.2f} ms/step, kernel span {span / a.steps:.2f} ms/step "
          f"over {a.steps} steps ({len(win) / a.steps:.0f} kernels/step)\n")
    print("| ms/step | % | launches/step | kernel |\n|---:|---:|---:|---|")
    for n, t in sorted(tot.items(), key=lambda kv: -kv[1])[:a.top]:
        print(f"| {t / a.steps:.3f} | {100 * t / busy:.1f} | {cnt[n] / a.steps:.1f} | `{n[:110]}` |")


if __name__ == "__main__":
    main()
