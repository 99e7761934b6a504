"""Where a kernel's scratch frame is used: per function of a hipcc object's gfx950 code object,
the scratch instructions and the line span they occupy, and the calls (s_swappc) a kernel makes.

usage: python tools/scratch_report.py spark-timeseries_amd/build/arima_cg_p2_s1.o [symbol-substring ...]
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def disassemble(obj):
    with tempfile.TemporaryDirectory() as td:
        subprocess.check_call([f"{LLVM}/llvm-objdump", "--offloading", os.path.abspath(obj)], cwd=td,
                              stdout=subprocess.DEVNULL)
        base = os.path.dirname(os.path.abspath(obj))
        dev = [f for f in os.listdir(base) if "amdgcn" in f and os.path.basename(obj) in f][0]
        path = os.path.join(base, dev)
        try:
            return subprocess.check_output([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", path], text=True)
        finally:
            os.remove(path)


def report(obj, filters):
    cur, funcs = None, {}
    for ln in disassemble(obj).splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", ln)
        if m:
            cur = m.group(1)
            funcs[cur] = dict(lines=0, scratch=[], calls=0)
            continue
        if cur is None or not ln.startswith("\t"):
            continue
        f = funcs[cur]
        f["lines"] += 1
        if "scratch_" in ln:
            f["scratch"].append(f["lines"])
        if "s_swappc" in ln:
            f["calls"] += 1
    for name, f in funcs.items():
        if filters and not any(x in name for x in filters):
            continue
        sc = f["scratch"]
        where = "-" if not sc else (f"lines {sc[0]}-{sc[-1]} of {f['lines']}" if len(sc) < 8 else
                                    f"first {sum(1 for x in sc if x <= 600)} in lines 1-600, last "
                                    f"{sum(1 for x in sc if x > f['lines'] - 600)} in the final 600 of {f['lines']}")
        print(f"{name[:90]:90s} scratch_ops={len(sc):4d} calls={f['calls']} {where}")


if __name__ == "__main__":
    report(sys.argv[1], sys.argv[2:])
