"""Build ``movie_recommender_amd/lib/cpp_ls_lib.so`` (hipcc, gfx950 only)."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")


def build(jobs=4, verbose=False):
    jobs = max(1, min(int(jobs), 16))
    cmd = ["make", "-C", CSRC, f"-j{jobs}"]
    r = subprocess.run(cmd, capture_output=not verbose, text=True)
    if r.returncode != 0:
        raise RuntimeError("HIP build failed:\n" + (r.stdout or "") + (r.stderr or ""))
    return os.path.join(HERE, "lib", "cpp_ls_lib.so")


if __name__ == "__main__":
    print(build(verbose=True))
