"""CallbackVerbose (ffddp.callbacks): the per-iteration lines the reference
prints with solver.setCallbacks([crocoddyl.CallbackVerbose()]) when
cfg.verbose is set (crocoddyl_classical.py:352-353, 360-361), from trace
records; and the oracle's records carry the same fields.  CPU only."""
import io

import numpy as np

from ffddp import _abi
from ffddp.callbacks import CallbackVerbose
from oracle import fddp

from test_oracle import _lqr


def _rows(n, max_it=12):
    t = np.full((max_it, _abi.TRACE_W), np.nan)
    for i in range(n):
        t[i] = [i, 1234.5 / (i + 1), 0.5 ** i, -3.25e2 / (i + 1), 1e-9 * 10 ** min(i, 3), 1e-9 * 10 ** min(i, 3),
                0.5 ** (i % 3), 50.0 / (i + 1), 7.0, 6.5]
    return t


def test_verbose_format_and_header_period():
    cb = CallbackVerbose(stream=io.StringIO())
    lines = cb.format(_rows(12))
    # header before iterations 0 and 10, one line per recorded iteration
    assert len(lines) == 14 and lines[0] == cb.header() and lines[11] == cb.header()
    assert lines[0].split() == ["iter", "cost", "stop", "grad", "preg", "dreg", "step", "||ffeas||", "||gfeas||",
                                "||hfeas||"]
    f = lines[1].split()
    assert f[0] == "0" and f[1] == "1.234e+03"  # precision 3 (1234.5 rounds half to even)
    assert float(f[3]) == -325.0 and f[6] == "1.0000" and float(f[7]) == 50.0 and float(f[8]) == 0.0
    assert lines[3].split()[6] == "0.2500"  # step length: 4 decimals
    # NaN rows (iterations not run) print nothing
    assert len(cb.format(_rows(3))) == 4


def test_verbose_callback_prints_one_instance():
    out = io.StringIO()
    cb = CallbackVerbose(level=2, instance=1, stream=out)
    tr = np.stack([_rows(2), _rows(5)])
    cb(None, tr)
    text = out.getvalue().splitlines()
    assert len(text) == 6 and "dV-exp" in text[0]
    assert float(text[1].split()[-1]) == 7.0 and float(text[1].split()[-2]) == 6.5  # level 2: dV-exp, dV
    assert cb.lines == text


def test_oracle_trace_fields():
    """The oracle records what the device trace records: one row per
    iteration with the accepted step's dV / dVexp and grad = -d1."""
    rng = np.random.default_rng(3)
    m = _lqr(rng)
    s = fddp.SolverBoxFDDP(m, box=False, consts=fddp.Consts(neg_step_rule=1))
    s.solve(np.zeros((m.N + 1, m.nx)), np.zeros((m.N, m.nu)), maxiter=10)
    tr = np.array(s.trace)
    assert tr.shape == (s.iter + 1, _abi.TRACE_W)
    assert np.array_equal(tr[:, 0], np.arange(s.iter + 1))
    assert tr[0, 7] > 0 and tr[-1, 7] == 0.0  # ||ffeas||: gaps closed by the full step
    assert tr[-1, 1] == s.cost and tr[-1, 2] == s.stop
    lines = CallbackVerbose(stream=io.StringIO()).format(tr)
    assert len(lines) == s.iter + 2
