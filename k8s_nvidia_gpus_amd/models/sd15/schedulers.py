"""Noise schedulers for SD1.5 sampling: PNDM (PLMS, SD1.5's default), DDIM, Euler (discrete).

Formulas follow the published samplers as diffusers implements them for SD1.5's
``scheduler_config.json`` (scaled-linear betas 0.00085→0.012 over 1000 steps, ``steps_offset=1``,
``set_alpha_to_one=False``, ``skip_prk_steps=True``, ε-prediction).  The reference pipeline uses the
checkpoint's PNDM scheduler (reference sd15-api/configmap.yaml:41: ``from_pretrained`` defaults).

Schedulers keep their per-step coefficients as Python floats and update latents with a handful of
fused elementwise ops, so the UNet's HIP graph (pipeline.py) stays free of scheduler state.
"""
from __future__ import annotations

from typing import List, Optional

import torch

from .config import SchedulerConfig


def alphas_cumprod(cfg: SchedulerConfig) -> torch.Tensor:
    n = cfg.num_train_timesteps
    if cfg.beta_schedule == "scaled_linear":
        betas = torch.linspace(cfg.beta_start ** 0.5, cfg.beta_end ** 0.5, n,
                               dtype=torch.float32) ** 2
    elif cfg.beta_schedule == "linear":
        betas = torch.linspace(cfg.beta_start, cfg.beta_end, n, dtype=torch.float32)
    else:
        raise ValueError(cfg.beta_schedule)
    return torch.cumprod(1.0 - betas, dim=0)


class _Base:
    init_noise_sigma = 1.0

    def __init__(self, cfg: SchedulerConfig = SchedulerConfig()):
        self.cfg = cfg
        self.alphas_cumprod = alphas_cumprod(cfg).double()
        self.final_alpha_cumprod = 1.0 if cfg.set_alpha_to_one else float(self.alphas_cumprod[0])
        self.timesteps: List[int] = []
        self.num_inference_steps = 0

    def _leading(self, n: int) -> List[int]:
        ratio = self.cfg.num_train_timesteps // n
        return [int(i * ratio + self.cfg.steps_offset) for i in range(n)][::-1]

    def _acp(self, t: int) -> float:
        return float(self.alphas_cumprod[t]) if t >= 0 else self.final_alpha_cumprod

    def scale_model_input(self, x: torch.Tensor, t: int) -> torch.Tensor:
        return x


class PNDMScheduler(_Base):
    """Pseudo linear multistep (PLMS) with SD1.5's ``skip_prk_steps``."""

    def set_timesteps(self, n: int) -> None:
        self.num_inference_steps = n
        ratio = self.cfg.num_train_timesteps // n
        base = [int(i * ratio + self.cfg.steps_offset) for i in range(n)]
        plms = base[:-1] + base[-2:-1] + base[-1:]
        self.timesteps = plms[::-1]
        self.ets: List[torch.Tensor] = []
        self.counter = 0
        self.cur_sample: Optional[torch.Tensor] = None

    def _prev(self, sample, t, prev_t, eps):
        a_t, a_prev = self._acp(t), self._acp(prev_t)
        b_t, b_prev = 1.0 - a_t, 1.0 - a_prev
        sample_coeff = (a_prev / a_t) ** 0.5
        denom = a_t * b_prev ** 0.5 + (a_t * b_t * a_prev) ** 0.5
        return sample_coeff * sample - ((a_prev - a_t) / denom) * eps

    def step(self, eps: torch.Tensor, t: int, sample: torch.Tensor) -> torch.Tensor:
        ratio = self.cfg.num_train_timesteps // self.num_inference_steps
        prev_t = t - ratio
        if self.counter != 1:
            self.ets = self.ets[-3:]
            self.ets.append(eps)
        else:
            prev_t = t
            t = t + ratio
        e = self.ets
        if len(e) == 1 and self.counter == 0:
            self.cur_sample = sample
            out_eps = eps
        elif len(e) == 1 and self.counter == 1:
            out_eps = (eps + e[-1]) * 0.5
            sample = self.cur_sample
            self.cur_sample = None
        elif len(e) == 2:
            out_eps = (3 * e[-1] - e[-2]) * 0.5
        elif len(e) == 3:
            out_eps = (23 * e[-1] - 16 * e[-2] + 5 * e[-3]) / 12
        else:
            out_eps = (55 * e[-1] - 59 * e[-2] + 37 * e[-3] - 9 * e[-4]) / 24
        self.counter += 1
        return self._prev(sample, t, prev_t, out_eps)


class DDIMScheduler(_Base):
    """Deterministic DDIM (η = 0)."""

    def set_timesteps(self, n: int) -> None:
        self.num_inference_steps = n
        self.timesteps = self._leading(n)

    def step(self, eps: torch.Tensor, t: int, sample: torch.Tensor) -> torch.Tensor:
        prev_t = t - self.cfg.num_train_timesteps // self.num_inference_steps
        a_t, a_prev = self._acp(t), self._acp(prev_t)
        x0 = (sample - (1 - a_t) ** 0.5 * eps) / a_t ** 0.5
        return a_prev ** 0.5 * x0 + (1 - a_prev) ** 0.5 * eps


class EulerDiscreteScheduler(_Base):
    """Euler sampler on the σ parameterisation (``timestep_spacing="leading"`` like SD1.5)."""

    def set_timesteps(self, n: int) -> None:
        self.num_inference_steps = n
        self.timesteps = self._leading(n)
        acp = self.alphas_cumprod
        sig = [float(((1 - acp[t]) / acp[t]) ** 0.5) for t in self.timesteps]
        self.sigmas = sig + [0.0]
        self.init_noise_sigma = (max(sig) ** 2 + 1) ** 0.5
        self._i = 0

    def scale_model_input(self, x: torch.Tensor, t: int) -> torch.Tensor:
        s = self.sigmas[self.timesteps.index(t)]
        return x / ((s ** 2 + 1) ** 0.5)

    def step(self, eps: torch.Tensor, t: int, sample: torch.Tensor) -> torch.Tensor:
        i = self.timesteps.index(t)
        return sample + (self.sigmas[i + 1] - self.sigmas[i]) * eps


SCHEDULERS = {"pndm": PNDMScheduler, "ddim": DDIMScheduler, "euler": EulerDiscreteScheduler}


def make_scheduler(name: str, cfg: SchedulerConfig = SchedulerConfig()):
    try:
        return SCHEDULERS[name.lower()](cfg)
    except KeyError:
        raise ValueError(f"unknown scheduler {name!r} (have {sorted(SCHEDULERS)})") from None
