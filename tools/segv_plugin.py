"""pytest plugin (-p segv_plugin with tools/ on PYTHONPATH): install the native backtrace
handler of tools/libsegv_trace.so before the tests run (use with -p no:faulthandler)."""
import ctypes
import os

_lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libsegv_trace.so"))
assert _lib.segv_trace_install() == 0
