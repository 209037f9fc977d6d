"""Mirror of gnark's backend.ProverOption / ProverConfig (backend/backend.go:57-137).

gnark selects the GPU path with ``backend.WithIcicleAcceleration()`` which sets
``ProverConfig.Accelerator = "icicle"`` (backend.go:132-137); the icicle prover
then checks ``opt.Accelerator`` (icicle.go:141-143).  This backend uses the
accelerator name ``"amd"``; ``with_icicle_acceleration`` is kept as an alias so
call sites written for the icicle path select the MI355X backend unchanged.
"""
from __future__ import annotations

import dataclasses
from typing import Callable, List, Optional

ACCELERATOR = "amd"


@dataclasses.dataclass
class ProverConfig:
    solver_opts: list = dataclasses.field(default_factory=list)
    hash_to_field_fn: Optional[object] = None
    challenge_hash: Optional[object] = None
    kzg_folding_hash: Optional[object] = None
    accelerator: str = ""


ProverOption = Callable[[ProverConfig], None]


def new_prover_config(*opts: ProverOption) -> ProverConfig:
    """backend.NewProverConfig (backend.go:70-83)."""
    cfg = ProverConfig()
    for o in opts:
        o(cfg)
    return cfg


def with_solver_options(*solver_opts) -> ProverOption:
    def f(cfg):
        cfg.solver_opts = list(solver_opts)
    return f


def with_amd_acceleration() -> ProverOption:
    def f(cfg):
        cfg.accelerator = ACCELERATOR
    return f


def with_icicle_acceleration() -> ProverOption:
    """Alias of backend.WithIcicleAcceleration (backend.go:132-137)."""
    return with_amd_acceleration()


def accelerated(cfg: ProverConfig) -> bool:
    return cfg.accelerator in (ACCELERATOR, "icicle")
