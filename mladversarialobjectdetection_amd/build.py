"""Build libphx.so in-tree for gfx950 (hipcc; no CMake).  `python -m mladversarialobjectdetection_amd.build`"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def build(jobs: int = 8, verbose: bool = False) -> str:
    csrc = os.path.join(HERE, "csrc")
    env = dict(os.environ)
    cmd = ["make", "-C", csrc, f"-j{min(jobs, 16)}"]
    r = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if verbose or r.returncode != 0:
        sys.stdout.write(r.stdout)
    if r.returncode != 0:
        raise RuntimeError("libphx build failed")
    return os.path.join(HERE, "libphx.so")


if __name__ == "__main__":
    print(build(verbose=True))
