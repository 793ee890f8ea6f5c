#!/usr/bin/env python3
"""Does the x2f16 GEMM lose fp16-subnormal plane values?  (Diagnostic.)

The activation split writes plane 1 = fp16(16 a - fp16(16 a)); for small |a|
that low plane (and for tiny |a| plane 0 too) is an fp16 subnormal.  This runs
the engine's planar GEMM (tvr_gemm_planar, v_mfma_f32_16x16x32_f16) on one
row whose activations are chosen so that one plane is subnormal and the other
zero or normal, against W = 1, and prints what the matrix core returned
against the exact value — 0 where subnormal inputs are flushed."""
import json
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import tvr_amd  # noqa: E402

X2F16 = tvr_amd._lib.GEMM_MODES["x2f16"]


def run(a_vals):
    lib = tvr_amd._lib.load()
    st = torch.cuda.current_stream().cuda_stream
    K = 64
    A = torch.zeros(1, K)
    A[0, :len(a_vals)] = torch.tensor(a_vals)
    W = torch.ones(1, K)
    scale = float(2.0 ** (15 - int(np.frexp(1.0)[1])))
    planes = torch.empty(2, 1, K, dtype=torch.int16, device="cuda")
    tvr_amd._lib.check(lib.tvr_weight_planes(X2F16, W.cuda().data_ptr(), scale, planes.data_ptr(), K, st), "w")
    Ad = A.cuda()
    Ah = torch.empty(1, 2, K, dtype=torch.int16, device="cuda")
    flag = torch.zeros(1, dtype=torch.int32, device="cuda")
    tvr_amd._lib.check(lib.tvr_act_rows(X2F16, Ad.data_ptr(), K, Ah.data_ptr(), 1, K, flag.data_ptr(), st), "a")
    C = torch.empty(1, 1, device="cuda")
    tvr_amd._lib.check(lib.tvr_gemm_planar(X2F16, Ah.data_ptr(), K, planes.data_ptr(), K, K, scale, 0, C.data_ptr(),
                                           1, 1, 1, K, st), "gemm")
    torch.cuda.synchronize()
    p = Ah.view(torch.float16).cpu().double()[0]
    return C.item(), float(A.double().sum()), p[0, :len(a_vals)].tolist(), p[1, :len(a_vals)].tolist()


cases = {
    "a = 1 (both planes normal)": [1.0],
    "a = 1 + 2^-15 (plane 1 = 2^-11 * ... normal)": [1.0 + 2.0 ** -15],
    "a = 1 + 2^-22 (plane 1 subnormal)": [1.0 + 2.0 ** -22],
    "a = 2^-24 (plane 0 subnormal, 16a = 2^-20)": [2.0 ** -24],
    "a = 3e-3 (plane 1 subnormal?)": [3e-3],
    "64 x 3e-6": [3e-6] * 64,
}
for name, vals in cases.items():
    c, exact, p0, p1 = run(vals)
    print(json.dumps({"case": name, "gemm": c, "exact": exact, "rel_err": abs(c - exact) / abs(exact),
                      "plane0": p0[:2], "plane1": p1[:2]}))
