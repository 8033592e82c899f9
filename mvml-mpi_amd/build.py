"""Build libmvml_gat.so in-tree with hipcc for gfx950 (no cmake, no torch extension).

    python mvml-mpi_amd/build.py            # incremental (objects newer than sources kept)
    python mvml-mpi_amd/build.py --clean
"""
import argparse
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(HERE, "build")
OUT = os.path.join(HERE, "mvml_gat", "libmvml_gat.so")
HEADER = os.path.join(HERE, "..", "include", "mvml_gat.h")
ARCH = os.environ.get("MVML_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function",
         "-Wno-unused-variable", "-Wno-unused-result"]


def sources():
    return sorted(f for f in os.listdir(CSRC) if f.endswith((".hip", ".cpp")))


def _stale(obj, deps):
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(d) > t for d in deps)


def compile_one(src):
    path = os.path.join(CSRC, src)
    obj = os.path.join(OBJ, src + ".o")
    deps = [path, HEADER] + [os.path.join(CSRC, h) for h in os.listdir(CSRC) if h.endswith(".h")]
    if not _stale(obj, deps):
        return obj
    cmd = [HIPCC, *FLAGS, "-c", path, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
    return obj


def build(clean=False, jobs=4):
    if clean and os.path.isdir(OBJ):
        shutil.rmtree(OBJ)
    os.makedirs(OBJ, exist_ok=True)
    with ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(compile_one, sources()))
    if _stale(OUT, objs):
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", OUT + ".tmp"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
        os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("-j", type=int, default=4)
    a = ap.parse_args()
    print(build(a.clean, a.j))
    sys.exit(0)
