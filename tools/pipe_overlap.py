"""Dev tool: how the kernels of a pipelined bench run overlap, from a rocprofv3 kernel trace.

usage: python tools/pipe_overlap.py <run_kernel_trace.csv | results.db> [--skip-first N]

Prints, per kernel family (k_cg_fit, k_hr_init, k_difference, ...): dispatches, summed duration, and the share of that
duration during which at least one k_cg_fit dispatch was running (HR or differencing work hidden under fits vs on its
own); and the share of the traced span with no fit kernel running at all.
"""
import argparse
import csv
import re
import sqlite3


def load(path):
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        return [(n, int(s), int(e)) for n, s, e in c.execute("select name, start, end from kernels")]
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            out.append((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    return out


def family(name):
    return re.sub(r"<.*", "", name.split("(")[0]).replace("void ", "").strip()


def union(iv):
    iv = sorted(iv)
    out = []
    for s, e in iv:
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def overlap(s, e, merged):
    tot = 0
    for a, b in merged:
        if b <= s:
            continue
        if a >= e:
            break
        tot += min(b, e) - max(a, s)
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--skip-first", type=int, default=0, help="ignore dispatches before the N-th k_cg_fit (warmup)")
    a = ap.parse_args()
    ks = sorted(load(a.trace), key=lambda x: x[1])
    fits = [k for k in ks if family(k[0]).endswith("k_cg_fit")]
    t0 = fits[a.skip_first][1] if a.skip_first and len(fits) > a.skip_first else ks[0][1]
    ks = [k for k in ks if k[1] >= t0]
    fits = [k for k in ks if family(k[0]).endswith("k_cg_fit")]
    fm = union([[s, e] for _, s, e in fits])
    span = max(e for _, _, e in ks) - min(s for _, s, _ in ks)
    fam = {}
    for n, s, e in ks:
        d = fam.setdefault(family(n), [0, 0, 0])
        d[0] += 1
        d[1] += e - s
        d[2] += overlap(s, e, fm)
    print(f"span {span / 1e6:.1f} ms, fit kernels running {sum(b - a for a, b in fm) / span:.3f} of it")
    for k, (n, dur, ov) in sorted(fam.items(), key=lambda x: -x[1][1]):
        print(f"{k:36s} n={n:5d} sum={dur / 1e6:10.2f} ms  under a fit {ov / max(dur, 1):.3f}")


if __name__ == "__main__":
    main()
