"""Print per-kernel VGPR/AGPR/SGPR/scratch of a hipcc object (dev tool).

usage: python tools/kernel_resources.py spark-timeseries_amd/build/arima_kernels.o [name-filter ...]
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def kernels(obj):
    with tempfile.TemporaryDirectory() as td:
        subprocess.check_call([f"{LLVM}/llvm-objdump", "--offloading", os.path.abspath(obj)], cwd=td,
                              stdout=subprocess.DEVNULL)
        dev = [f for f in os.listdir(os.path.dirname(os.path.abspath(obj))) if "amdgcn" in f and
               os.path.basename(obj) in f]
        base = os.path.dirname(os.path.abspath(obj))
        path = os.path.join(base, dev[0])
        notes = subprocess.check_output([f"{LLVM}/llvm-readelf", "--notes", path], text=True)
        for f in os.listdir(base):
            if ".o.0." in f:
                os.remove(os.path.join(base, f))
    out = []
    for blk in re.split(r"\n  - \.agpr_count:", notes)[1:]:
        name = re.search(r"\.name:\s+(\S+)", blk).group(1)
        get = lambda k: int(re.search(r"\." + k + r":\s+(\d+)", blk).group(1))
        out.append(dict(name=name, agpr=int(blk.split("\n")[0].strip()), vgpr=get("vgpr_count"),
                        sgpr=get("sgpr_count"), scratch=get("private_segment_fixed_size")))
    return out


if __name__ == "__main__":
    flt = sys.argv[2:]
    for k in kernels(sys.argv[1]):
        if not flt or any(f in k["name"] for f in flt):
            print(f"{k['name'][:70]:70s} vgpr={k['vgpr']:4d} agpr={k['agpr']:4d} sgpr={k['sgpr']:4d} "
                  f"scratch={k['scratch']}")
