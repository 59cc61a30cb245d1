#!/usr/bin/env python3
"""Diagnostic: run bench.py in a process that imported torch first (so
libuwvk.so binds to torch's bundled HIP runtime), optionally with a CUDA
context made by torch.  usage: python tools/bench_with_torch.py [--ctx] -- <bench args>"""
import os
import runpy
import sys

ctx = "--ctx" in sys.argv
args = sys.argv[sys.argv.index("--") + 1:] if "--" in sys.argv else []
import torch  # noqa: E402,F401
if ctx:
    torch.zeros(1, device="cuda")
maps = sorted({l.split()[-1] for l in open("/proc/self/maps") if "amdhip64" in l})
print("libamdhip64 mapped before bench:", maps, file=sys.stderr)
sys.argv = ["bench.py"] + args
runpy.run_path(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py"),
               run_name="__main__")
