"""Run the VGPR-resident lite-pass timing prototype (csrc/dsr_proto.hip) beside the shipped kernel's
numbers from the same box (VERDICT r3 item 4's kill criterion: keep only at >= +8 %
over the shipped lite kernel's one-stream rate).  Prints one JSON line.
    python tools/proto_vres.py [tiles] [reps]"""
import ctypes as C
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = C.CDLL(os.path.join(REPO, "dsp-slam-rgbd_amd", "csrc", "libdsr_proto.so"))
tiles = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
out = {}
for t in (256, 1024, tiles):
    tf, ms, cs = C.c_float(), C.c_float(), C.c_float()
    rc = lib.dsr_proto_vres(0, t, reps, C.byref(tf), C.byref(ms), C.byref(cs))
    out[f"tiles_{t}"] = {"rc": rc, "tflops": round(tf.value, 1), "ms_per_launch": round(ms.value, 4),
                         "checksum": cs.value}
print(json.dumps(out))
