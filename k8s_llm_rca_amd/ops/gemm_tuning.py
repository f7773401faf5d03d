"""Tuned hipBLASLt/rocBLAS solutions for the decode-bucket projection GEMMs.

``tools/tune_gemms.py`` times every library solution (PyTorch TunableOp) for
the (M, N, K) shapes that pure-decode HIP-graph steps run -- M is one of the
engine's graph batch buckets -- and writes ``data/gemm_tuned_<model>.csv``.
:func:`load` enables TunableOp *read-only*: listed shapes use their measured
winner, every other shape the default heuristic, nothing is tuned online.
Measured on MI355X (profiles/r1_gemm_tunableop_8b.txt): per-shape wins of up
to ~35 % (down projection, M = 128-192) but losses elsewhere (3 % net over the
decode buckets), so it is off by default (``K8SRCA_GEMM_TUNING=1``); the
measured dispatch of :mod:`.linear` (hand-written gemm_mid / skinny kernels
vs hipBLASLt per shape) is the default path.
"""
from __future__ import annotations

from ..knobs import KNOBS
import logging
import os
import shutil
import tempfile
from typing import Optional

import torch

log = logging.getLogger(__name__)

DATA_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "data")
_loaded: Optional[str] = None


def table_path(model: str, tp: int = 1) -> str:
    return os.path.join(DATA_DIR, f"gemm_tuned_{model}" + (f"-tp{tp}" if tp > 1 else "") + ".csv")


def load(model: str, tp: int = 1) -> bool:
    """Use the tuned GEMM table of ``model`` at TP degree ``tp`` if one exists
    for this build (TunableOp validators: torch / HIP / hipBLASLt / arch)."""
    global _loaded
    if not KNOBS.gemm_tuning or not torch.cuda.is_available():
        return False
    path = table_path(model, tp)
    if _loaded == path:
        return True
    if not os.path.exists(path):
        return False
    T = torch.cuda.tunable
    # TunableOp writes its results file at exit: point it at a scratch copy so
    # the shipped table is never rewritten
    scratch = os.path.join(tempfile.gettempdir(), f"k8srca_tunableop_{os.getpid()}.csv")
    shutil.copyfile(path, scratch)
    T.set_filename(scratch, insert_device_ordinal=False)
    T.tuning_enable(False)
    T.record_untuned_enable(False)
    T.enable(True)
    ok = T.read_file(scratch)
    if not ok:
        log.warning("GEMM tuning table %s does not match this build; using default heuristics", path)
        T.enable(False)
        return False
    _loaded = path
    return True
