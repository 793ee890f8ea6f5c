"""Library fp16 / bf16 GEMM throughput at the engine's shapes (a ceiling probe).

Times ``torch.matmul`` (hipBLASLt / rocBLAS underneath) on fp16 and bf16
operands with fp32 accumulation at the two C3 GEMM shapes, with K as the
engine sees it and with K tripled (the three split products of x2f16 written
as one plain GEMM over [a0 | a1 | a0] x [w0 | w0 | w1]).  Output: one JSON
line per case, TFLOP/s of the plain library GEMM and of the fp32-equivalent
work when K is tripled.  Diagnostic only; nothing in the engine calls it.
"""
import json
import sys

import torch


def time_mm(a, b, iters):
    for _ in range(2):
        torch.matmul(a, b.t())
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        torch.matmul(a, b.t())
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 90000
    d, dm = 2560, 10240
    shapes = {"qkv_mlpin": (3 * d + dm, d), "o_mlpout": (d, d + dm)}
    out = []
    for dt in (torch.float16, torch.bfloat16):
        for name, (N, K) in shapes.items():
            for kmul in (1, 3):
                a = torch.randn(M, K * kmul, device="cuda", dtype=dt)
                w = torch.randn(N, K * kmul, device="cuda", dtype=dt)
                ms = time_mm(a, w, 5)
                tf = 2.0 * M * N * K * kmul / ms / 1e9
                rec = {"dtype": str(dt).split(".")[-1], "shape": name, "M": M, "N": N, "K": K * kmul,
                       "ms": round(ms, 3), "tflops": round(tf, 1)}
                if kmul == 3:
                    rec["fp32_equiv_tflops"] = round(tf / 3, 1)
                print(json.dumps(rec), flush=True)
                out.append(rec)
                del a, w
                torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
