"""The drop-in's `_cg_status` bookkeeping (iterative_solver.py:874-965) replayed per device chunk
(solvers/iterative_solver.py `_CGStatus._replay`) against the reference's per-call recurrence,
restated here call by call: same num_iters, resid, eff, history and summed call time for any
split of the iterations into chunks.  CPU only."""
import collections

import numpy as np
import pytest

from sgdml_amd.solvers.iterative_solver import _CGStatus


class _PerCall:
    """iterative_solver.py:874-918, one scipy callback at a time."""

    def __init__(self, iters0):
        self.num_iters, self.resid, self.avg_tt, self.calls = iters0, 0.0, 0.0, 0
        self.hist = collections.deque(maxlen=100)
        self.eff = 0

    def call(self, resid, tt, last):
        self.avg_tt += 0.0 if self.calls == 0 else tt
        old, self.resid = self.resid, resid
        self.hist.append(0.0 if self.num_iters == 0 else self.resid - old)
        h = np.asarray(self.hist)
        tot = np.abs(h).sum()
        ratio = (-h.clip(max=0).sum() / tot) if tot > 0 else 1
        self.eff = 0 if self.num_iters == 0 else (int(100 * ratio) - 50) * 2
        self.calls += 1
        if not last:
            self.num_iters += 1


@pytest.mark.parametrize("iters0", [0, 37])
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_replay_matches_per_call(iters0, seed):
    rng = np.random.default_rng(seed)
    m = 700
    trace = np.exp(np.cumsum(rng.normal(-0.01, 0.05, m + 1)))
    cuts = np.unique(np.concatenate([[0, m], rng.choice(np.arange(1, m), 12, replace=False),
                                     [1, 2, 101, 102]]))
    st = _CGStatus.__new__(_CGStatus)
    st.num_iters, st.resid, st.avg_tt, st.calls, st.eff = iters0, 0.0, 0.0, 0, 0
    st.hist = collections.deque(maxlen=_CGStatus.HIST_LEN)
    ref = _PerCall(iters0)
    for c, (j0, j1) in enumerate(zip(cuts[:-1], cuts[1:])):
        tt = 1e-3 * (c + 1)
        st._replay(trace, int(j0), int(j1), tt)
        for j in range(j0 + 1, j1 + 1):
            ref.call(float(trace[j]), tt, j == j1)
        assert st.num_iters == ref.num_iters and st.eff == ref.eff
        assert st.resid == ref.resid and st.calls == ref.calls
        assert list(st.hist) == list(ref.hist)
        assert st.avg_tt == ref.avg_tt
        # the caller increments num_iters after the chunk's last call (run())
        st.num_iters += 1
        ref.num_iters += 1
