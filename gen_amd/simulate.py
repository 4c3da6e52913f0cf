"""simulate(model, args) over libgen_hip.so (gh_simulate).

`simulate(gen_fn, args)` (src/gen_fn_interface.jl:149; Static IR
src/static_ir/simulate.jl:23-34,50-83; the Unfold's
src/modeling_library/unfold/simulate.jl) samples every choice of the model
and records each choice's score.  Here one call simulates `num_traces`
independent traces on the GPU; trace i is a function of (seed, i) only.
"""
from __future__ import annotations

import numpy as np

from . import _lib
from .choicemap import ChoiceMap, Selection, select as _select
from .models import DiscreteHMM, Model


class SimulatedTraces:
    """num_traces traces of simulate(model, (T,)): time-major columns
    xs [T, d, n], ys [T, dy, n], per-step scores [T, 2, n] (latent, observation)
    and get_score [n]."""

    def __init__(self, model: Model, T: int, xs, ys, per_step, total):
        self.model, self.T = model, T
        self.xs, self.ys, self.per_step, self.total = xs, ys, per_step, total

    def __len__(self):
        return self.total.size

    def __getitem__(self, i) -> "SimulatedTrace":
        i = int(i)
        if not -len(self) <= i < len(self):
            raise IndexError(i)
        return SimulatedTrace(self, i % len(self))

    def _locate(self, addr):
        """(kind, t, component slice) of a choice address."""
        m, a = self.model, tuple(addr)
        if m.static:
            if a == ("slope",):
                return "x", 1, 0
            if a == ("intercept",):
                return "x", 1, 1
            for i in range(1, m.dy + 1):
                if a == tuple(m.y_address(i)):
                    return "y", 1, i - 1
            raise KeyError(addr)
        for t in range(1, self.T + 1):
            las = [tuple(la) for la in m.latent_addresses(t)]
            if a in las:
                return "x", t, (None if len(las) == 1 else ("part", las.index(a)))
            if a == tuple(m.obs_address(t)):
                return "y", t, None
        raise KeyError(addr)

    def column(self, addr) -> np.ndarray:
        """The value of `addr` in every trace: [n] for a scalar choice, [n, k] for a vector."""
        kind, t, comp = self._locate(addr)
        src = self.xs if kind == "x" else self.ys
        col = src[t - 1]
        if isinstance(comp, tuple):  # one of several latent addresses
            return self.model.latent_part_column(comp[1], col.T)
        if comp is not None:
            return col[comp]
        if isinstance(self.model, DiscreteHMM):
            return col[0].astype(np.int64)
        return col[0] if col.shape[0] == 1 else col.T


class SimulatedTrace:
    """One simulated trace, with the accessors of src/gen_fn_interface.jl."""

    def __init__(self, traces: SimulatedTraces, i: int):
        self.traces, self.i = traces, i

    def __getitem__(self, addr):
        return self.traces.column(addr)[self.i]

    def get_args(self) -> tuple:
        tr = self.traces
        return () if tr.model.static else (tr.T,)

    def get_gen_fn(self) -> Model:
        return self.traces.model

    def get_score(self) -> float:
        return float(self.traces.total[self.i])

    def get_choices(self) -> ChoiceMap:
        tr, m, i = self.traces, self.traces.model, self.i
        cm = ChoiceMap()
        if m.static:
            cm[("slope",)] = float(tr.xs[0, 0, i])
            cm[("intercept",)] = float(tr.xs[0, 1, i])
            for r in range(m.dy):
                cm[m.y_address(r + 1)] = float(tr.ys[0, r, i])
            return cm
        for t in range(1, tr.T + 1):
            x, y = tr.xs[t - 1, :, i], tr.ys[t - 1, :, i]
            las = m.latent_addresses(t)
            if len(las) > 1:
                for k, la in enumerate(las):
                    cm[la] = m.latent_part(k, x)
            else:
                cm[m.latent_address(t)] = _value(m, x)
            cm[m.obs_address(t)] = _value(m, y)
        return cm

    def project(self, selection) -> float:
        """project(trace, selection) (src/static_ir/project.jl:8-28): the summed
        scores of the selected choices; the static model's :slope and
        :intercept share one latent score column and are not separable there."""
        tr, m, i = self.traces, self.traces.model, self.i
        sel = selection if isinstance(selection, Selection) else _select(*selection)
        total = 0.0
        for a in sel:
            kind, t, comp = tr._locate(a)
            if m.static and comp is not None and kind == "x":
                mu, sd = (m.mu_s, m.sd_s) if comp == 0 else (m.mu_i, m.sd_i)
                v = sd * sd
                x = tr.xs[0, comp, i]
                total += -((x - mu) ** 2) / (2.0 * v) - 0.5 * np.log(2.0 * np.pi * v)
            elif m.static and kind == "y":
                x0, x1 = tr.xs[0, 0, i], tr.xs[0, 1, i]
                v = m.sigma * m.sigma
                y = tr.ys[0, comp, i]
                total += -((y - (x0 * m.xs[comp] + x1)) ** 2) / (2.0 * v) - 0.5 * np.log(2.0 * np.pi * v)
            else:
                total += tr.per_step[t - 1, 0 if kind == "x" else 1, i]
        return float(total)


def _value(m: Model, v: np.ndarray):
    if isinstance(m, DiscreteHMM):
        return int(v[0])
    return float(v[0]) if v.size == 1 else v.copy()


def simulate(model: Model, model_args: tuple = (), num_traces: int | None = None, seed: int = 0, ctx=None):
    """simulate(model, model_args): model_args = (T,) for the Unfold models, ()
    for the static regression.  Returns one trace, or with num_traces = n a
    SimulatedTraces batch of n traces simulated in one launch."""
    from .pf import default_context

    U = None
    if model.static:  # its argument (the xs) is part of the model object
        T = 1
    else:
        if getattr(model, "inputs", False) and len(model_args) == 2:  # (T, U): a slot model's per-step inputs
            U = np.ascontiguousarray(np.asarray(model_args[1], dtype=np.float64).reshape(int(model_args[0]), model.d))
            model_args = model_args[:1]
        if len(model_args) != 1:
            raise _lib.GenHipError(1, "simulate: model_args = (T,) for an Unfold model, (T, U) with per-step inputs")
        T = int(model_args[0])
    n = 1 if num_traces is None else int(num_traces)
    ctx = ctx or default_context()
    h = ctx.model_handle(model)
    vec = model.family in (_lib.FAMILY_LGSSM, _lib.FAMILY_REGRESSION, _lib.FAMILY_SLOTS)
    d, dy = (model.d, model.dy) if vec else (1, 1)
    xs, ys = np.empty((T, d, n)), np.empty((T, dy, n))
    ps, tot = np.empty((T, 2, n)), np.empty(n)
    if U is not None:
        _lib.check(_lib.load().gh_simulate_inputs(h, T, n, int(seed), _lib.dptr(U), _lib.dptr(xs), _lib.dptr(ys),
                                                  _lib.dptr(ps), _lib.dptr(tot)))
    else:
        _lib.check(_lib.load().gh_simulate(h, T, n, int(seed), _lib.dptr(xs), _lib.dptr(ys), _lib.dptr(ps),
                                           _lib.dptr(tot)))
    out = SimulatedTraces(model, T, xs, ys, ps, tot)
    return out[0] if num_traces is None else out
