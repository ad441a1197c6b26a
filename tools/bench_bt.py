"""bench.py in this process with a native backtrace on a host fault
(tools/native/segv_bt.c) and Python's faulthandler: where a crash sits.
usage: python tools/bench_bt.py [bench.py arguments]"""
import ctypes
import faulthandler
import os
import runpy
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
import torch  # noqa: E402,F401  (these imports replace signal handlers: ours go in after them)
sys.path.insert(0, os.path.join(HERE, ".."))
import pluss_sampler_optimization_amd  # noqa: E402,F401
torch.cuda.set_device(0)
faulthandler.enable()
bt = ctypes.CDLL(os.path.join(HERE, "native", "libsegv_bt.so"))
assert bt.segv_bt_install() == 0
sys.argv = [os.path.join(HERE, "..", "bench.py")] + sys.argv[1:]
runpy.run_path(sys.argv[0], run_name="__main__")
