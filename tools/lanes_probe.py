"""Does running two CIE sweeps concurrently (two engine instances, two HIP
streams, two host threads) raise throughput over one?  Diagnostic only.

    python tools/lanes_probe.py [steps]
"""
import json
import sys
import threading
import time

import torch

sys.path.insert(0, ".")
import tvr_amd  # noqa: E402
from tvr_amd.experiments import causal_indirect_effect_sums  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    dev = torch.device("cuda", 0)
    cfg = tvr_amd.get_config("pythia-2.8b")
    models = [tvr_amd.Model.from_pretrained("pythia-2.8b", device=dev, seed=0, gemm="x2f16") for _ in range(2)]
    g = torch.Generator(device=dev).manual_seed(4321)
    mean = torch.randn(cfg.n_layers, cfg.n_heads, cfg.d_model, device=dev, generator=g) * 0.5
    prompts = [tvr_amd.prompts.synthetic_cie_prompts(m, 12, 4, seed=1234 + i) for i, m in enumerate(models)]
    streams = [torch.cuda.Stream(dev) for _ in models]

    def run(i, n):
        with torch.cuda.stream(streams[i]):
            for _ in range(n):
                causal_indirect_effect_sums(mean, prompts[i][0], prompts[i][1], models[i])
            streams[i].synchronize()

    run(0, 1)
    run(1, 1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(0, steps)
    t1 = time.perf_counter() - t0
    single = 12 * cfg.n_layers * cfg.n_heads * steps / t1
    th = [threading.Thread(target=run, args=(i, steps)) for i in range(2)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    t2 = time.perf_counter() - t0
    dual = 2 * 12 * cfg.n_layers * cfg.n_heads * steps / t2
    print(json.dumps({"single_lane_patched_prompts_per_s": round(single, 1), "two_lanes": round(dual, 1),
                      "ratio": round(dual / single, 3), "steps": steps}))


if __name__ == "__main__":
    main()
