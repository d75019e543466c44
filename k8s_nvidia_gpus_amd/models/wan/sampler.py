"""Flow-matching sigma schedules and samplers for Wan2.1 (the ``KSampler`` node of the reference's
ComfyUI graph: ``sampler_name=uni_pc, scheduler=simple``, generate_wan_t2v.py:305-312).

Conventions (ComfyUI's ``ModelSamplingDiscreteFlow`` for Wan, shift 8):

* training grid ``σ(t) = s·t / (1 + (s−1)·t)``, ``t = i/1000``, i = 1…1000; the model's timestep
  input is ``1000·σ``;
* the network predicts the velocity ``v = ε − x₀``; ``x_σ = (1−σ)·x₀ + σ·ε``, so the denoised
  estimate is ``x₀ = x − σ·v``;
* schedulers ``simple`` (every (1000/steps)-th training sigma from the top), ``normal`` and
  ``sgm_uniform`` (uniform in timestep, mapped through the shift), all ending at σ = 0.

Samplers: ``euler`` (first-order flow ODE), ``uni_pc`` / ``uni_pc_bh2`` (UniPC multistep
predictor–corrector, order 2, data prediction, B(h) = h or eᵸ−1), run in the flow
parameterisation (α = 1−σ, log-SNR λ = log α − log σ) as Wan's own release does.  ComfyUI's uni_pc
runs its VE-form conversion on the same sigmas; outputs therefore differ slightly from a ComfyUI
render with the same seed ("parity unpinned": no reference render exists offline).
"""
from __future__ import annotations

import math
from typing import Callable, List, Optional

import torch

Denoiser = Callable[[torch.Tensor, float], torch.Tensor]   # (x, sigma) -> x0 estimate


def flow_sigma(t: torch.Tensor, shift: float) -> torch.Tensor:
    return shift * t / (1 + (shift - 1) * t)


def training_sigmas(shift: float, n: int = 1000) -> torch.Tensor:
    return flow_sigma(torch.arange(1, n + 1, dtype=torch.float64) / n, shift)


def schedule(name: str, steps: int, shift: float, denoise: float = 1.0) -> torch.Tensor:
    """σ_0 > … > σ_{steps−1} > σ_steps = 0 (float64).  ``denoise < 1`` keeps the last
    ``steps`` sigmas of a ``steps/denoise`` schedule (ComfyUI's partial-denoise convention)."""
    if steps < 1:
        raise ValueError("steps must be >= 1")
    total = steps if denoise >= 1.0 else int(steps / max(denoise, 1e-4))
    sig = training_sigmas(shift)
    if name == "simple":
        ss = len(sig) / total
        s = [float(sig[-(1 + int(i * ss))]) for i in range(total)]
    elif name == "normal":
        t_hi, t_lo = float(sig[-1]) * 1000.0, float(sig[0]) * 1000.0
        ts = torch.linspace(t_hi, t_lo, total, dtype=torch.float64)
        # ComfyUI's flow sampling maps timestep→σ through the shift again (σ(ts) = shift(ts/1000))
        s = [float(flow_sigma(x / 1000.0, shift)) for x in ts]
    elif name == "sgm_uniform":
        t_hi, t_lo = float(sig[-1]) * 1000.0, float(sig[0]) * 1000.0
        ts = torch.linspace(t_hi, t_lo, total + 1, dtype=torch.float64)[:-1]
        s = [float(flow_sigma(x / 1000.0, shift)) for x in ts]
    else:
        raise ValueError(f"unknown scheduler {name!r} (simple | normal | sgm_uniform)")
    out = torch.tensor(s + [0.0], dtype=torch.float64)
    return out[-(steps + 1):]


SAMPLERS = ("euler", "uni_pc", "uni_pc_bh2")
SCHEDULERS = ("simple", "normal", "sgm_uniform")


def sample_euler(model: Denoiser, x: torch.Tensor, sigmas: torch.Tensor,
                 callback=None) -> torch.Tensor:
    for i in range(len(sigmas) - 1):
        s, s1 = float(sigmas[i]), float(sigmas[i + 1])
        x0 = model(x, s)
        x = x + (s1 - s) * (x - x0) / s
        if callback:
            callback(i, x0)
    return x


def _lam(s: float) -> float:
    """log-SNR λ = log((1−σ)/σ); σ = 1 (pure noise, λ = −∞) is clamped to 1 − 10⁻⁴ so the first
    UniPC step keeps a finite B(h)."""
    s = min(max(s, 1e-12), 1.0 - 1e-4)
    return math.log(1.0 - s) - math.log(s)


def _coeffs(hs: List[float], h: float, order: int, bh2: bool):
    """UniPC's (R, b, B(h), φ₁) for data prediction: ``hs`` are the normalised past step
    offsets r_k = (λ_k − λ_s0)/h of the extra history points."""
    hh = -h
    h_phi_1 = math.expm1(hh)
    h_phi_k = h_phi_1 / hh - 1.0
    fact = 1
    b_h = math.expm1(hh) if bh2 else hh
    rks = list(hs) + [1.0]
    R, b = [], []
    for j in range(1, order + 1):
        R.append([r ** (j - 1) for r in rks])
        b.append(h_phi_k * fact / b_h)
        fact *= j + 1
        h_phi_k = h_phi_k / hh - 1.0 / fact
    return R, b, b_h, h_phi_1


def sample_unipc(model: Denoiser, x: torch.Tensor, sigmas: torch.Tensor, bh2: bool = False,
                 order: int = 2, callback=None) -> torch.Tensor:
    """UniPC-p / UniC multistep (order ≤ 2 predictor, corrector on every step but the last), one
    model evaluation per step; the final step to σ = 0 is first order (returns the x₀ estimate)."""
    hist: List[tuple] = []            # (sigma, lambda, x0)
    x_prev: Optional[torch.Tensor] = None
    prev_order = 1
    n = len(sigmas) - 1
    for i in range(n):
        s = float(sigmas[i])
        m = model(x, s)
        if callback:
            callback(i, m)
        lam_t = _lam(s)
        if x_prev is not None:                          # UniC: refine x at σ_i with m
            s0, l0, m0 = hist[-1]
            h = lam_t - l0
            hs, d1 = [], []
            for k in range(1, prev_order):
                _, lk, mk = hist[-(k + 1)]
                rk = (lk - l0) / h
                hs.append(rk)
                d1.append((mk - m0) / rk)
            R, b, b_h, phi1 = _coeffs(hs, h, prev_order, bh2)
            if prev_order == 1:
                rhos = [0.5]
            else:
                rhos = torch.linalg.solve(torch.tensor(R, dtype=torch.float64),
                                          torch.tensor(b, dtype=torch.float64)).tolist()
            alpha_t = 1.0 - s
            xt_ = (s / s0) * x_prev - alpha_t * phi1 * m0
            corr = sum(r * d for r, d in zip(rhos[:-1], d1)) if d1 else 0.0
            x = xt_ - alpha_t * b_h * (corr + rhos[-1] * (m - m0))
        hist.append((s, lam_t, m))
        hist = hist[-order:]
        s_next = float(sigmas[i + 1])
        if s_next <= 0.0:
            return m                                    # first-order step to σ = 0
        cur_order = min(order, len(hist))
        if i == n - 2 and n < 10:
            cur_order = min(cur_order, 2)
        l_next = _lam(s_next)
        h = l_next - lam_t
        hs, d1 = [], []
        for k in range(1, cur_order):
            _, lk, mk = hist[-(k + 1)]
            rk = (lk - lam_t) / h
            hs.append(rk)
            d1.append((mk - m) / rk)
        R, b, b_h, phi1 = _coeffs(hs, h, cur_order, bh2)
        alpha_n = 1.0 - s_next
        x_prev = x
        xt_ = (s_next / s) * x - alpha_n * phi1 * m
        if d1:
            if cur_order == 2:
                rhos_p = [0.5]
            else:
                rhos_p = torch.linalg.solve(torch.tensor(R, dtype=torch.float64)[:-1, :-1],
                                            torch.tensor(b, dtype=torch.float64)[:-1]).tolist()
            x = xt_ - alpha_n * b_h * sum(r * d for r, d in zip(rhos_p, d1))
        else:
            x = xt_
        prev_order = cur_order
    return x


def sample(name: str, model: Denoiser, x: torch.Tensor, sigmas: torch.Tensor, callback=None):
    if name == "euler":
        return sample_euler(model, x, sigmas, callback)
    if name in ("uni_pc", "uni_pc_bh2"):
        return sample_unipc(model, x, sigmas, bh2=name.endswith("bh2"), callback=callback)
    raise ValueError(f"unknown sampler {name!r} ({' | '.join(SAMPLERS)})")


def initial_noise(seed: int, shape, sigma_max: float) -> torch.Tensor:
    """ComfyUI's convention: CPU ``torch.manual_seed(seed)`` Gaussian noise, scaled by σ_max
    (flow noise scaling of an empty latent)."""
    g = torch.Generator(device="cpu").manual_seed(int(seed) & 0xFFFFFFFFFFFFFFFF)
    return torch.randn(tuple(shape), generator=g, dtype=torch.float32) * sigma_max
