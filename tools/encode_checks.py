#!/usr/bin/env python3
"""Diagnostic: run the frame-assembly GPU tests against the range-checked build
(tools/libnetc_ws_gpu_checks.so, -DNETC_ENC_CHECKS) and report the first access that
would have left its buffer (site, value, limit, count)."""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = os.path.join(ROOT, "tools", "libnetc_ws_gpu_checks.so")
env = dict(os.environ, NETC_GPU_LIB=lib)
code = ("import ctypes, sys, pytest\n"
        "rc = pytest.main(['-q', '-x', 'tests/test_gpu_encode.py'] + sys.argv[1:])\n"
        "from netc_amd import _lib\n"
        "out = (ctypes.c_ulonglong * 4)()\n"
        "_lib.gpu().netc_gpu_debug_encode_faults(out)\n"
        "print('ENC_FAULT site=%d value=%d limit=%d count=%d' % tuple(out))\n"
        "sys.exit(rc)\n")
sys.exit(subprocess.call([sys.executable, "-c", code] + sys.argv[1:], env=env, cwd=ROOT))
