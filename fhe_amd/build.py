"""In-tree build of the native library (hipcc --offload-arch=gfx950)."""
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))


def build(jobs=8, verbose=False):
    cmd = ["make", "-C", os.path.join(_HERE, "csrc"), f"-j{jobs}"]
    r = subprocess.run(cmd, capture_output=not verbose, text=True)
    if r.returncode != 0:
        raise RuntimeError("fhe_amd native build failed:\n" + (r.stdout or "") + (r.stderr or ""))
    return os.path.join(_HERE, "libfhe_amd.so")
