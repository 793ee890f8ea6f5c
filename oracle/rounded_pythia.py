"""ORACLE (test infrastructure only) — the layer-streamed fp64 oracle with
selected intermediates ROUNDED to a narrower type, the way a GEMM path rounds
them: fp32 (what the reference's own fp32 arithmetic does), bf16 / fp16 (the
engine's 16-bit GEMM operands: weights, LayerNorm outputs, z, GELU(h), the
final norm's output).  It measures how much error a rounding scheme alone
produces at full depth — the floor any implementation of that arithmetic
has — so the bf16 parity test can hold the engine to "no more than its own
operand roundings explain" (tests/test_gpu_full_depth.py), and
tools/precision_probe.py can rank the rounding points.  Everything not
rounded stays fp64; the rounding points follow csrc/ (split.hpp store_ln4: the
bf16 mode's Q / K operands are fp16, the rest bf16).
"""
from __future__ import annotations

import math

import torch

from .streamed_pythia import StreamedPythiaOracle


def r16(x, dtype):
    """Round to a 16-bit type; fp16 with a power-of-two scale into its range (as the engine's planes)."""
    if dtype == torch.bfloat16:
        return x.to(torch.bfloat16).to(x.dtype)
    m = x.abs().max().item()
    s = 2.0 ** (14 - math.ceil(math.log2(m))) if m > 0 else 1.0
    return (x * s).to(torch.float16).to(x.dtype) / s


class Rounded(StreamedPythiaOracle):
    """fp64 streamed oracle with rounding points.  ``rules``: name -> callable(x)."""

    def __init__(self, cfg, get_raw, rules):
        self.rules = rules
        super().__init__(cfg, get_raw)
        self._wcache = {}

    def R(self, name, x):
        f = self.rules.get(name)
        return f(x) if f else x

    def block(self, l):
        b = super().block(l)
        if self._wcache.get("l") != l:
            self._wcache = {"l": l, "w": {k: self.R("w_" + k, v) for k, v in b.items()}}
        return self._wcache["w"]

    def _ln_pre(self, x):
        x = self.R("ln_in", x)
        y = super()._ln_pre(x)
        return self.R("ln_out", y)

    def _block(self, l, resid, replace=(), add_last=(), want_result_last=False):
        w = self.block(l)
        x = self._ln_pre(resid)
        xq = self.R("a_qk", x)
        xv = self.R("a_v", x)
        q = self._rotate(self.R("gemm_out", torch.einsum("bpd,hde->bphe", xq, w["W_Q"]) + w["b_Q"]))
        k = self._rotate(self.R("gemm_out", torch.einsum("bpd,hde->bphe", xq, w["W_K"]) + w["b_K"]))
        v = self.R("gemm_out", torch.einsum("bpd,hde->bphe", xv, w["W_V"]) + w["b_V"])
        T = x.shape[1]
        scores = self.R("attn", torch.einsum("bqhe,bkhe->bhqk", q, k) / math.sqrt(self.cfg.d_head))
        mask = torch.triu(torch.ones(T, T, dtype=torch.bool, device=x.device), diagonal=1)
        pat = self.R("attn", torch.softmax(scores.masked_fill(mask, float("-inf")), dim=-1))
        z = self.R("attn", torch.einsum("bkhe,bhqk->bqhe", v, pat))
        H, dh, d = self.cfg.n_heads, self.cfg.d_head, self.cfg.d_model
        zo = self.R("a_z", z)
        acc = self.rules.get("acc")  # (splits of the O + MLP-out GEMM, splits of the others) or None
        if acc and not replace and not add_last:
            # the engine's fused GEMMs with fp32 accumulation: [Q|K|V|MLP-in] = xn W1^T, [O|MLP-out] over
            # K = d + d_mlp in one accumulator (csrc/engine.hip run_block / run_block_out)
            b_ = z.shape[0]
            W1 = torch.cat([w["W_Q"].permute(1, 0, 2).reshape(d, H * dh), w["W_K"].permute(1, 0, 2).reshape(d, H * dh),
                            w["W_V"].permute(1, 0, 2).reshape(d, H * dh), w["W_in"]], 1)
            y = self.acc_matmul(xv.reshape(b_ * T, d), W1, splits=acc[1]).reshape(b_, T, -1)
            qa = self._rotate((y[..., :d].reshape(b_, T, H, dh) + w["b_Q"]).float().double())
            ka = self._rotate((y[..., d:2 * d].reshape(b_, T, H, dh) + w["b_K"]).float().double())
            va = (y[..., 2 * d:3 * d].reshape(b_, T, H, dh) + w["b_V"]).float().double()
            sc = torch.einsum("bqhe,bkhe->bhqk", qa, ka) / math.sqrt(dh)
            za = torch.einsum("bkhe,bhqk->bqhe", va, torch.softmax(sc.masked_fill(mask, float("-inf")), dim=-1))
            za = self.R("a_z", za.float().double())
            ga = self.R("a_gelu", torch.nn.functional.gelu((y[..., 3 * d:] + w["b_in"]).float().double()).float().double())
            W2 = torch.cat([w["W_O"].reshape(H * dh, d), w["W_out"]], 0)
            o = self.acc_matmul(torch.cat([za.reshape(b_, T, H * dh), ga], -1).reshape(b_ * T, -1), W2,
                                splits=acc[0]).reshape(b_, T, d)
            res_last = torch.einsum("bhe,hed->bhd", za[:, -1], w["W_O"]) if want_result_last else None
            return (resid + (o + (w["b_O"] + w["b_out"]))).float().double(), res_last
        attn = self.R("gemm_out", zo.reshape(z.shape[0], T, H * dh) @ w["W_O"].reshape(H * dh, d))
        if replace and self.rules.get("entry_engine"):
            # the engine's REPLACE_HEAD entry (csrc/entry_mfma.hpp): the clean row's attention output as the
            # rounded GEMM computed it, minus the replaced head's z_h W_O[h] in fp32 operands (the trace's z
            # and the fp32 W_O), plus the vector — instead of re-summing the other heads' rounded products
            raw = StreamedPythiaOracle.block(self, l)["W_O"]
            for r, h, vec in replace:
                attn[r] = attn[r] - z[r, :, h, :].float().double() @ raw[h].float().double() + vec.to(attn)
        elif replace:
            rows = sorted({r for r, _, _ in replace})
            ri = torch.tensor(rows, device=x.device)
            result = torch.einsum("bqhe,hed->bqhd", zo[ri], w["W_O"])
            at = {r: i for i, r in enumerate(rows)}
            for r, h, vec in replace:
                result[at[r], :, h, :] = vec.to(result)
            attn[ri] = result.sum(-2)
        for r, vec in add_last:
            attn[r, -1] = attn[r, -1] + vec.to(attn)
        h = self.R("gemm_out", xv @ w["W_in"] + w["b_in"])
        g = self.R("a_gelu", torch.nn.functional.gelu(h))
        mlp = self.R("gemm_out", g @ w["W_out"])
        res_last = torch.einsum("bhe,hed->bhd", z[:, -1], w["W_O"]) if want_result_last else None
        return self.R("resid", resid + (attn + w["b_O"]) + (mlp + w["b_out"])), res_last

    @staticmethod
    def _hi(x, scale):
        return (x * scale).float().half().double() / scale

    def acc_matmul(self, x, w, step=32, splits=1, three=None):
        """x @ w the way a matrix core accumulates it in fp32 (rule "acc"): products of 32-deep k-slices exact,
        each slice added to an fp32 accumulator (one rounding per slice), ``splits`` K ranges accumulated
        separately and summed in fp32 at the end (split-K).  x: [..., K] (already rounded operands)."""
        K = x.shape[-1]
        three = self.rules.get("acc3") if three is None else three
        if three:  # the x2f16 GEMM's three products per slice, small terms first (csrc/gemm_pingpong.hpp)
            m = w.abs().max().item()
            sw = 2.0 ** (14 - math.floor(math.log2(m))) if m > 0 else 1.0
            x0, w0 = self._hi(x, 16.0), self._hi(w, sw)
            parts = [(x - x0, w0), (x0, w - w0), (x0, w0)]
        else:
            parts = [(x, w)]
        out = None
        for s in range(splits):
            k0, k1 = s * K // splits, (s + 1) * K // splits
            acc = torch.zeros(x.shape[:-1] + (w.shape[-1],), dtype=torch.float32, device=x.device)
            for k in range(k0, k1, step):
                for xa, wa in parts:
                    acc = (acc.double() + xa[..., k:min(k + step, k1)] @ wa[k:min(k + step, k1)]).float()
            out = acc if out is None else (out.double() + acc.double()).float()
        return out.double()

    def _final_last(self, resid):
        x = self.R("a_u", self._ln_pre(resid[:, -1]))
        if self.rules.get("acc"):
            return self.acc_matmul(x, self.R("w_U", self.W_U)) + self.b_U
        return x @ self.R("w_U", self.W_U) + self.b_U


def x2f16(x):
    """The engine's fp32-accurate split (csrc/split.hpp): s x = fp16(s x) + fp16(s x - fp16(s x)), s a power of
    two putting max |x| in fp16's range; the value the three-product GEMM sees (22 significand bits)."""
    m = x.abs().max().item()
    s = 2.0 ** (14 - math.ceil(math.log2(m))) if m > 0 else 1.0
    y = (x * s).float()
    h0 = y.half().float()
    h1 = (y - h0).half().float()
    return (h0.double() + h1.double()) / s


def _ftz16(h):
    """fp16 values below the smallest normal (2^-14) flushed to zero."""
    return torch.where(h.abs() < 2.0 ** -14, torch.zeros_like(h), h)


def x2f16_act(x, scale=16.0, ftz=False):
    """The engine's activation split (csrc/split.hpp): a fixed scale (X2_ASCALE = 16), fp16(16 a) +
    fp16(16 a - fp16(16 a)); ``ftz``: fp16 subnormals read as zero (as a matrix core that flushes them)."""
    y = (x * scale).float()
    h0 = y.half().float()
    h1 = (y - h0).half().float()
    if ftz:
        h0, h1 = _ftz16(h0), _ftz16(h1)
    return (h0.double() + h1.double()) / scale


def x2f16_weight(x, ftz=False):
    """The weight planes: one power-of-two scale per matrix putting max |W| in [2^14, 2^15]."""
    m = x.abs().max().item()
    s = 2.0 ** (14 - math.floor(math.log2(m))) if m > 0 else 1.0
    y = (x * s).float()
    h0 = y.half().float()
    h1 = (y - h0).half().float()
    if ftz:
        h0, h1 = _ftz16(h0), _ftz16(h1)
    return (h0.double() + h1.double()) / s


F32 = lambda x: x.float().double()  # noqa: E731
BF = lambda x: r16(x, torch.bfloat16)  # noqa: E731
FH = lambda x: r16(x, torch.float16)  # noqa: E731
WEIGHTS = ["w_W_Q", "w_W_K", "w_W_V", "w_W_O", "w_W_in", "w_W_out", "w_U"]
ACTS = ["a_qk", "a_v", "a_z", "a_gelu", "a_u"]


def variants():
    v = {"fp64": {},
         "fp32_all": {k: F32 for k in ["ln_in", "ln_out", "gemm_out", "attn", "resid", "a_gelu"] + WEIGHTS},
         "resid32": {"resid": F32}, "ln32": {"ln_in": F32, "ln_out": F32}, "attn32": {"attn": F32},
         "gemm32": {"gemm_out": F32}, "gelu32": {"a_gelu": F32}, "w32": {k: F32 for k in WEIGHTS}}
    allbf = {k: BF for k in WEIGHTS + ACTS}
    v["all_bf16"] = allbf
    eng = dict(allbf, a_qk=FH, w_W_Q=FH, w_W_K=FH)
    v["engine_bf16"] = eng
    # + the engine's REPLACE_HEAD entry form (clean attention output - z_h W_O[h] + vector, fp32 operands)
    v["engine_bf16_entry"] = dict(eng, entry_engine=True)
    v["w_bf16"] = {k: BF for k in WEIGHTS}
    v["act_bf16"] = {k: BF for k in ACTS}
    v["all_f16"] = {k: FH for k in WEIGHTS + ACTS}
    # the x2f16 GEMM path: every GEMM operand split into two fp16 planes, the rest of the arithmetic fp32
    v["x2f16_ops"] = {k: x2f16 for k in WEIGHTS + ACTS}
    v["x2f16_engine"] = dict(v["fp32_all"], **{k: x2f16 for k in WEIGHTS + ACTS})
    # the engine's split exactly: activations at the fixed scale 16, weights per matrix; with and without
    # fp16 subnormals; and a larger activation scale
    for tag, fa, fw in (("x2e", lambda x: x2f16_act(x), x2f16_weight),
                        ("x2e_ftz", lambda x: x2f16_act(x, ftz=True), lambda x: x2f16_weight(x, ftz=True)),
                        ("x2e_a256", lambda x: x2f16_act(x, 256.0), x2f16_weight),
                        ("x2e_a256_ftz", lambda x: x2f16_act(x, 256.0, True), lambda x: x2f16_weight(x, ftz=True))):
        v[tag] = dict(v["fp32_all"], **{k: fw for k in WEIGHTS}, **{k: fa for k in ACTS})
        v[tag + "_acts_only"] = {k: fa for k in ACTS}
        v[tag + "_gelu_only"] = {"a_gelu": fa}
    # plus the matrix cores' fp32 accumulation (32-deep slices, one rounding each; clean forwards only):
    # the whole K in one accumulator, or the O + MLP-out GEMM split in 2 / 4
    for sp in (1, 2, 4):
        v[f"x2e_acc_o{sp}"] = dict(v["x2e"], acc=(sp, 1))
        v[f"x2e_acc3_o{sp}"] = dict(v["x2e"], acc=(sp, 1), acc3=True)
    v["fp32_acc"] = dict(v["fp32_all"], acc=(1, 1))
    for k in WEIGHTS + ACTS:  # the engine's bf16 mode with ONE operand group kept exact
        v["engine_bf16_but_" + k] = {kk: vv for kk, vv in eng.items() if kk != k}
    return v
