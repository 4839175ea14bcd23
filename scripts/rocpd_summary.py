"""Summarise a rocprofv3 ``--kernel-trace`` database (rocpd sqlite, the default
output of ``rocprofv3 -d DIR -o run``) as markdown: per-kernel ms/step, % of
GPU-busy time, launches/step and stream; GPU-busy and kernel-span per step.

    python scripts/rocpd_summary.py gpurun_out/prof/run_results.db --steps 5 \
        --title "..." > profiles/xxx.md

``--steps`` is the number of steps to attribute; the window is the last
``--steps`` occurrences of ``--marker`` x ``--per-step`` (default: the fused
SGD kernel, once per gradient bucket) — or the whole trace with ``--all``.
"""
import argparse
import collections
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--marker", default="sgd_flat_kernel")
    ap.add_argument("--per-step", type=int, default=5)
    ap.add_argument("--all", action="store_true")
    ap.add_argument("--title", default="")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--detail", default="",
                    help="also list every launch (one step) of kernels containing this text, "
                         "with its duration and the kernel that ran before it")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, stream_id, start, end from kernels order by start").fetchall()
    if not rows:
        raise SystemExit("no kernels in trace")
    lo, hi = rows[0][2], rows[-1][3]
    if not a.all:
        marks = [r for r in rows if a.marker in r[0]]
        need = a.steps * a.per_step
        if len(marks) < need + 1:
            raise SystemExit(f"only {len(marks)} '{a.marker}' launches, need {need + 1}")
        lo = marks[-need - 1][3]          # end of the last marker before the window
        hi = marks[-1][3]
    win = [r for r in rows if r[2] >= lo and r[3] <= hi]
    steps = a.steps if not a.all else 1
    tot = collections.defaultdict(float)
    cnt = collections.Counter()
    streams = collections.defaultdict(set)
    for n, s, t0, t1 in win:
        tot[n] += (t1 - t0) / 1e6
        cnt[n] += 1
        streams[n].add(s)
    busy = sum(tot.values())
    span = (hi - lo) / 1e6
    if a.title:
        print(f"# {a.title}\n")
    print(f"GPU busy {busy / steps:.2f} ms/step, kernel span {span / steps:.2f} ms/step over "
          f"{steps} steps ({len(win) / steps:.0f} kernels/step)\n")
    print("| ms/step | % | launches/step | stream | kernel |\n|---:|---:|---:|---|---|")
    for n, v in sorted(tot.items(), key=lambda kv: -kv[1])[:a.top]:
        nm = n if len(n) <= 110 else n[:107] + "..."
        print(f"| {v / steps:.3f} | {100 * v / busy:.1f} | {cnt[n] / steps:.1f} | "
              f"{','.join(map(str, sorted(streams[n])))} | `{nm}` |")

    if a.detail:
        per = len(win) // max(steps, 1)
        last = win[-per:]
        print(f"\n## Launches of `{a.detail}` in the last step\n")
        print("| us | previous kernel |\n|---:|---|")
        for i, (n, s_, t0, t1) in enumerate(last):
            if a.detail in n:
                prev = last[i - 1][0] if i else "-"
                prev = prev if len(prev) <= 90 else prev[:87] + "..."
                print(f"| {(t1 - t0) / 1e3:.1f} | `{prev}` |")

if __name__ == "__main__":
    main()

