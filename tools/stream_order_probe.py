"""Runs tools/stream_order_probe.hip (GPU box): same-stream producer -> consumer
pairs, with and without a second stream loading every CU, counting consumers that saw a stale
token (started before their producer's last workgroup finished).
Build: make -C dsp-slam-rgbd_amd/csrc tools   ->  tools/libstream_order.so"""
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(HERE, "libstream_order.so"))
lib.stream_order_probe.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_longlong, ctypes.c_int, ctypes.c_longlong,
                                   ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
iters = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
bad = 0
for grid in (256, 4096):
    for delay in (0, 100, 2000):                     # ticks of 100 MHz: 0, 1 us, 20 us
        for load in (0, 1):
            stale = ctypes.c_int(0)
            rc = lib.stream_order_probe(iters, grid, delay, load, 20000, 256 * 8, ctypes.byref(stale))
            print(f"grid {grid:5d} delay {delay / 100:5.1f} us load {load}: {'ERROR' if rc else stale.value} of {iters} "
                  f"consumers saw a stale token", flush=True)
            bad += rc != 0 or stale.value != 0
print("stream order held everywhere" if bad == 0 else f"{bad} settings with stale tokens or errors")
