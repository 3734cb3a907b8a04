"""HBM rate of the PPO update's memory-bound MLP ops at the 65 536-env mini-batch (393 216 rows, h = 256): gr_mlp_in
forward / backward (d = 16 inputs read from packed 44-float sample rows), gr_head forward / backward (k = 4 actor,
k = 1 critic).  HIP events around 20 back-to-back calls each; GB/s of the bytes each op must move.  GR_LIB_PATH picks
a variant library (scripts/build_patched.py).

    python scripts/time_update_kernels.py [--rows 393216] [--out file.json]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from generalizableracing_amd import _abi  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=393216)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    lib = _abi.load()
    dev = "cuda:0"
    m, h, d, ldx, slope = a.rows, 256, 16, 44, 0.01
    g = torch.Generator(device=dev).manual_seed(0)
    xs = torch.randn(m, ldx, device=dev, generator=g)
    w1 = torch.randn(h, d, device=dev, generator=g) * 0.3
    b1 = torch.randn(h, device=dev, generator=g) * 0.1
    h1 = torch.empty(m, h, device=dev)
    gh = torch.randn(m, h, device=dev, generator=g)
    z = torch.randn(m, h, device=dev, generator=g)
    gz = torch.empty(m, h, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    res = {"rows": m, "lib": os.environ.get("GR_LIB_PATH", "tree")}

    def timed(name, fn, nbytes):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.reps
        res[name] = {"us": us, "GBps": nbytes / (us * 1e-6) / 1e9}

    part_in = torch.empty(lib.gr_mlp_in_partials(m, d, h), device=dev)
    sums_in = torch.empty(h * d + h, device=dev)
    timed("in_forward", lambda: lib.gr_mlp_in_forward(xs.data_ptr(), m, d, ldx, w1.data_ptr(), b1.data_ptr(), h, slope,
                                                       h1.data_ptr(), st), m * (d * 4 + h * 4))
    timed("in_backward", lambda: lib.gr_mlp_in_backward(gh.data_ptr(), h1.data_ptr(), xs.data_ptr(), m, d, ldx, h, slope,
                                                         part_in.data_ptr(), sums_in.data_ptr(), st), m * (d * 4 + 2 * h * 4))
    for k in (4, 1):
        w3 = torch.randn(k, h, device=dev, generator=g) * 0.1
        b3 = torch.randn(k, device=dev, generator=g)
        y = torch.empty(m, k, device=dev)
        gy = torch.randn(m, k, device=dev, generator=g)
        part = torch.empty(lib.gr_head_partials(m, k, h), device=dev)
        sums = torch.empty(k * h + k + h, device=dev)
        timed(f"head_forward_k{k}", lambda: lib.gr_head_forward(z.data_ptr(), m, h, w3.data_ptr(), b3.data_ptr(), k, slope,
                                                                  y.data_ptr(), st), m * (h * 4 + k * 4))
        timed(f"head_backward_k{k}", lambda: lib.gr_head_backward(z.data_ptr(), gy.data_ptr(), m, h, w3.data_ptr(), k, slope,
                                                                    gz.data_ptr(), part.data_ptr(), sums.data_ptr(), st),
              m * (2 * h * 4 + k * 4))
    res["sum_us"] = sum(v["us"] for v in res.values() if isinstance(v, dict))
    # reference rates of the same matrix shape: torch's fill (write only) and copy (read + write)
    timed("ref_torch_fill", lambda: h1.fill_(1.0), m * h * 4)
    timed("ref_torch_copy", lambda: h1.copy_(gh), m * h * 8)
    print(json.dumps(res))
    if a.out:
        with open(a.out, "a") as f:
            f.write(json.dumps(res) + "\n")


if __name__ == "__main__":
    main()
