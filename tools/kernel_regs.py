"""VGPR / AGPR / spill / LDS usage of kernels in a built library (gfx950
code-object metadata), e.g.

    python tools/kernel_regs.py [--so PATH] [--match cg_onepass]
"""
import argparse
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_asm_guards import LLVM, SO, _gfx950_objects  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--so", default=SO)
    ap.add_argument("--match", default="cg_onepass")
    a = ap.parse_args()
    for obj in _gfx950_objects(a.so):
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(obj)
            f.flush()
            notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", f.name],
                                   capture_output=True, text=True).stdout
        for blk in notes.split("- .agpr_count")[1:]:
            name = re.search(r"\.name:\s+(\S+)", blk)
            if not name or a.match not in name.group(1):
                continue
            get = lambda k: (re.search(rf"\.{k}:\s+(\S+)", blk) or [None, "?"])[1]  # noqa: E731
            dem = subprocess.run(["c++filt", name.group(1)], capture_output=True,
                                 text=True).stdout.strip()
            agpr = blk.split("\n")[0].strip(": ")
            print(f"{dem[:90]:90s} vgpr {get('vgpr_count'):>4} agpr {agpr:>4} "
                  f"spill {get('vgpr_spill_count'):>3} lds {get('group_segment_fixed_size'):>6}")


if __name__ == "__main__":
    main()
