"""Time mimic_skb_prep_kernel variants in isolation (tools/prep_probe.sh builds them from skb.hip with
-D knobs): 1M IMIX sk_buff packets as the cfg-5 bench makes them, 20 launches between events."""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, ".")
from mimic_amd import workloads as W

# PREP_VARIETY: the fraction of header variants (the cfg-5 bench uses 0.05)
buf, off, lens = W.make_skb_packets(1 << 20, (64, 576, 1500), (7, 4, 1), variety=float(os.environ.get("PREP_VARIETY", "0")))
n = len(lens)
dev = torch.device("cuda:0")
d_buf = torch.from_numpy(buf).to(dev)
d_off = torch.from_numpy(off.view("int64")).to(dev)
d_len = torch.from_numpy(lens.view("int32")).to(dev)
rec = torch.empty(n * 160, dtype=torch.uint8, device=dev)
prefix = torch.empty(n + n // 256 + 1, dtype=torch.int64, device=dev)
state = torch.zeros(4, dtype=torch.int64, device=dev)
for so in sys.argv[1:] + ["norec:" + sys.argv[1]]:
    norec = so.startswith("norec:")
    lib = C.CDLL(so.split(":")[-1])
    f = lib.mimic_skb_prep_only
    f.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p]
    s = torch.cuda.current_stream()
    args = (d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n, None if norec else rec.data_ptr(), 12, prefix.data_ptr(),
            state.data_ptr(), C.c_void_p(s.cuda_stream))
    for _ in range(3):
        f(*args)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(20):
        f(*args)
    b.record()
    torch.cuda.synchronize()
    print(so, f"{a.elapsed_time(b) / 20 * 1000:.1f} us per launch", flush=True)
