"""ORACLE — test infrastructure only.

A CPU restatement (PyTorch on CPU, fp32 or fp64) of what the reference
computes, used as the CHECKER of the HIP engine:

* ``hooked_pythia`` — TransformerLens ``HookedTransformer`` semantics for Pythia
  (weight processing, hook points, ``run_with_cache`` / ``run_with_hooks`` /
  ``forward(start_at_layer=)``), written from TL's documented behaviour
   in TL's own 4-D weight layout, independently of the
  product's fused layout.
* ``reference_experiments`` — the reference's experiment functions restated
  line by line (scratch2.py / scratch.py), quirks included,
  driving the hooked model through Python hook callbacks exactly as the
  reference drives TransformerLens.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg
may import this package.  The product (``task-vector-replication_amd``) never
does, and has no CPU fallback.

Parity pinning: the forward is pinned against
HuggingFace ``transformers`` GPTNeoXForCausalLM on seeded weights
(``TL_logits == HF_logits - mean(HF_logits)``, softmax equal); the prompt
builders are pinned by fixtures generated from the reference's own functions
(tests/golden/make_prompt_fixtures.py).  TransformerLens itself is not
installed, so the per-head hook values (hook_result after fold_value_biases)
are pinned only by the App. A derivation: "parity partially unpinned" at the
TransformerLens hook boundary.
"""
