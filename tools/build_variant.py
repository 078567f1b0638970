"""Measurement build of libmmsbm.so with extra compile flags (A/B and stamp builds).

usage: python tools/build_variant.py OUT.so [-DFLAG=1 ...]   (e.g. tools/_build/libmmsbm_stamp.so -DMMSBM_STAMP=1)
"""
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from trigenicinteractionpredictor_amd import build  # noqa: E402

out = os.path.abspath(sys.argv[1])
os.makedirs(os.path.dirname(out), exist_ok=True)
cmd = build.command(out, extra=sys.argv[2:])
print(" ".join(cmd), file=sys.stderr)
subprocess.check_call(cmd)
