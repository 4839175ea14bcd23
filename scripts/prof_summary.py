"""Summarise a rocprofv3 kernel trace: steady-state per-step breakdown of the
last `--steps` steps (window = last steps*ms_per_step of the trace)."""
import argparse
import collections
import csv

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--steps", type=int, default=10)
ap.add_argument("--ms-per-step", type=float, required=True)
ap.add_argument("--top", type=int, default=40)
ap.add_argument("--md", default="")
ap.add_argument("--title", default="")
a = ap.parse_args()
rows = list(csv.DictReader(open(a.trace)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
end = int(rows[-1]["End_Timestamp"])
win = [r for r in rows if int(r["Start_Timestamp"]) > end - a.steps * a.ms_per_step * 1e6]
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in win)
agg = collections.defaultdict(lambda: [0, 0])
for r in win:
    k = r["Kernel_Name"][:110]
    agg[k][0] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    agg[k][1] += 1
lines = [f"GPU busy {busy / 1e6 / a.steps:.2f} ms/step over {a.steps} steps "
         f"({len(win) / a.steps:.0f} kernels/step)", "",
         "| ms/step | % | launches/step | kernel |", "|---:|---:|---:|---|"]
for k, (t, c) in sorted(agg.items(), key=lambda x: -x[1][0])[:a.top]:
    lines.append(f"| {t / 1e6 / a.steps:.3f} | {100 * t / busy:.1f} | {c / a.steps:.1f} | `{k}` |")
out = "\n".join(lines)
print(out)
if a.md:
    with open(a.md, "w") as f:
        f.write(f"# {a.title}\n\n{out}\n")
