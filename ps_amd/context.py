"""Process-wide run state (reference: context/Context.java).

The reference keeps run state in static volatile globals initialised from ``-D`` system
properties.  Here the same concepts live on one ``Context`` object (``ps_amd.context.ctx``):

  status        TRAINING / PREDICTING / LOSS_SURFACE_EVAL   (Context.java:14-16)
  mode          STANDALONE / DISTRIBUTED                    (Context.java:26-28)
  step          global step counter                         (Context.java:30)
  finish        early-stop flag set by models               (Context.java:22)
  weights_scale loss-surface interpolation factor           (Context.java:18)
  model_index   thread-local replica index                  (Context.java:12)

``is_report_ui()`` no longer dereferences an unset thread-local (fixes Q12: it returns True
for replica 0 and for any thread that never set an index).
"""
from __future__ import annotations

import enum
import threading

from .config import Config


class Stat(enum.Enum):
    TRAINING = "training"
    PREDICTING = "predicting"
    LOSS_SURFACE_EVAL = "loss_surface_eval"


class Mode(enum.Enum):
    STANDALONE = "standalone"
    DISTRIBUTED = "distributed"


class Context:
    def __init__(self, cfg: Config | None = None):
        self._local = threading.local()
        self._lock = threading.Lock()
        self.init(cfg)

    def init(self, cfg: Config | None = None) -> "Context":
        self.cfg = cfg or Config.from_env()
        self.mode = Mode.DISTRIBUTED if self.cfg.mode == "dist" else Mode.STANDALONE
        self.status = Stat.TRAINING
        self.weights_scale = 0.0
        self.finish = False
        self._step = 0
        return self

    # ------------------------------------------------------------- step counter
    @property
    def step(self) -> int:
        return self._step

    def incr_step(self) -> int:
        with self._lock:
            self._step += 1
            return self._step

    def set_step(self, v: int) -> None:
        """Resume: continue the global step counter from a checkpoint."""
        with self._lock:
            self._step = int(v)

    # ------------------------------------------------------------- replica index
    @property
    def model_index(self) -> int:
        return getattr(self._local, "model_index", 0)

    @model_index.setter
    def model_index(self, v: int) -> None:
        self._local.model_index = int(v)

    # ------------------------------------------------------------- predicates
    def is_training(self) -> bool:
        return self.status == Stat.TRAINING

    def is_report_ui(self) -> bool:
        if self.is_standalone():
            return self.model_index == 0
        return self.cfg.is_major and self.model_index == 0

    def is_pserver(self) -> bool:
        return self.cfg.ps

    def is_distributed(self) -> bool:
        return self.mode == Mode.DISTRIBUTED

    def is_standalone(self) -> bool:
        return self.mode == Mode.STANDALONE


ctx = Context()
