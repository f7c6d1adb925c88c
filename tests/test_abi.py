"""C-ABI: library loads on a CPU-only host, exports every declared symbol,
struct layouts agree with the header, host helpers agree with the oracle,
and API errors are reported (no compute on the device here)."""
import ctypes
import re
import subprocess
import tempfile
from pathlib import Path

import numpy as np

from ffddp import _abi
from oracle import panda as P

ROOT = Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "ffddp.h"


def declared_functions():
    txt = HEADER.read_text()
    return sorted(set(re.findall(r"^\s*(?:int|void|const char\*)\s+(ffddp_\w+)\s*\(", txt, re.M)))


def test_library_exports_every_declared_symbol():
    lib = _abi.load()
    names = declared_functions()
    assert len(names) >= 10
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) == set(_abi.SYMBOLS)


def test_struct_layout_matches_header():
    src = r'''
#include <stdio.h>
#include <stddef.h>
#include "ffddp.h"
int main(void) {
  printf("%zu %zu %zu %zu %d ", sizeof(ffddp_plant_params), offsetof(ffddp_plant_params, armature),
         offsetof(ffddp_plant_params, r_tool), offsetof(ffddp_plant_params, site_R), FFDDP_PLANT_OBS);
  printf("%zu %zu %zu %d %d %d ", sizeof(ffddp_solver_params), offsetof(ffddp_solver_params, reg_decfactor),
         offsetof(ffddp_solver_params, neg_step_rule), FFDDP_TRACE_W, FFDDP_NEGSTEP_CROCODDYL,
         FFDDP_NEGSTEP_BOUNDED_RISE);
  printf("%zu %zu %zu %d %d ", sizeof(ffddp_plan_io), offsetof(ffddp_plan_io, xs), offsetof(ffddp_plan_io, stats),
         FFDDP_NSTATS, FFDDP_NKERNELS);
  printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu %zu\n", sizeof(ffddp_robot), sizeof(ffddp_ocp_config),
         offsetof(ffddp_ocp_config, dt), offsetof(ffddp_ocp_config, R_des),
         offsetof(ffddp_ocp_config, y_weights), offsetof(ffddp_ocp_config, use_inner_tau_reg),
         sizeof(ffddp_task), offsetof(ffddp_task, has_ee_start), offsetof(ffddp_task, q_nom),
         offsetof(ffddp_task, torque_mode));
  return 0;
}'''
    with tempfile.TemporaryDirectory() as d:
        c = Path(d) / "t.c"
        c.write_text(src)
        exe = Path(d) / "t"
        subprocess.run(["gcc", "-I", str(ROOT / "include"), str(c), "-o", str(exe)], check=True)
        vals = [int(v) for v in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    C = _abi.OcpConfig
    Pp = _abi.PlantParams
    assert vals[:5] == [ctypes.sizeof(Pp), Pp.armature.offset, Pp.r_tool.offset, Pp.site_R.offset, _abi.PLANT_OBS]
    vals = vals[5:]
    Sp = _abi.SolverParams
    assert vals[:6] == [ctypes.sizeof(Sp), Sp.reg_decfactor.offset, Sp.neg_step_rule.offset, _abi.TRACE_W,
                        _abi.NEGSTEP_CROCODDYL, _abi.NEGSTEP_BOUNDED_RISE]
    assert len(_abi.TRACE_FIELDS) == _abi.TRACE_W
    vals = vals[6:]
    Pio = _abi.PlanIO
    assert vals[:5] == [ctypes.sizeof(Pio), Pio.xs.offset, Pio.stats.offset, _abi.NSTATS, len(_abi.KERNEL_CLASSES)]
    vals = vals[5:]
    assert vals == [
        ctypes.sizeof(_abi.Robot), ctypes.sizeof(C), C.dt.offset, C.R_des.offset, C.y_weights.offset,
        C.use_inner_tau_reg.offset, ctypes.sizeof(_abi.Task), _abi.Task.has_ee_start.offset, _abi.Task.q_nom.offset,
        _abi.Task.torque_mode.offset,
    ]


def test_host_helpers_match_oracle():
    rng = np.random.default_rng(0)
    q = P.Q_NEUTRAL + rng.uniform(-0.5, 0.5, size=(16, 7))
    assert np.allclose(_abi.gravity_torque(q), P.gravity_torque(q), rtol=0, atol=1e-12)
    for i in range(4):
        Rm, p = _abi.frame_placement(q[i])
        _, _, R2, p2 = P.forward_kinematics(q[i])
        assert np.allclose(Rm, R2, atol=1e-14) and np.allclose(p, p2, atol=1e-14)


def test_invalid_config_rejected_before_device():
    from ffddp.config import classical_preset

    lib = _abi.load()
    c = classical_preset(30).to_struct()
    c.nc = 2  # neither ContactModel1D nor 3D
    h = ctypes.c_void_p()
    rc = lib.ffddp_create(ctypes.byref(_abi.robot_struct()), ctypes.byref(c), 0, 4, ctypes.byref(h))
    assert rc == -1 and not h.value
    c = classical_preset(30).to_struct()
    rc = lib.ffddp_create(ctypes.byref(_abi.robot_struct()), ctypes.byref(c), 0, 0, ctypes.byref(h))
    assert rc == -1


def test_null_handle_errors():
    lib = _abi.load()
    assert lib.ffddp_profile_enable(None, 1) == -1
    assert b"null" in lib.ffddp_last_error(None)
    p = _abi.solver_params()
    assert lib.ffddp_get_solver_params(None, ctypes.byref(p)) == -1
    assert lib.ffddp_set_solver_params(None, ctypes.byref(p)) == -1
    assert lib.ffddp_trace_enable(None, 4) == -1
    assert lib.ffddp_trace_read(None, 1, None) == -1
    assert lib.ffddp_host_alloc(16, None) == -1
    assert lib.ffddp_host_free(None) == 0
    assert lib.ffddp_plan_create(None, 1, 10, 0, None, None) == -1
    assert lib.ffddp_plan_run(None) == -1
    lib.ffddp_plan_destroy(None)


def test_solver_param_defaults_match_oracle():
    """The library's SolverBoxFDDP defaults (mirrored by _abi.solver_params)
    are the oracle's constants (oracle/fddp.py Consts)."""
    from oracle import fddp

    c, p = fddp.Consts(), _abi.solver_params()
    assert p.th_stop == c.th_stop_box and _abi.solver_params(use_box=False).th_stop == c.th_stop_fddp
    for k in ("th_grad", "th_acceptstep", "th_acceptnegstep", "th_stepdec", "th_stepinc", "reg_min", "reg_max",
              "reg_incfactor", "reg_decfactor", "neg_step_rule"):
        assert getattr(p, k) == getattr(c, k), k
    hdr = HEADER.read_text()
    for k, v in (("th_stop", "5e-5"), ("th_grad", "1e-12"), ("th_acceptnegstep", "2.0")):
        assert re.search(rf"double {k};\s*/\*[^*]*{re.escape(v)}", hdr), k


def test_integration_snippet_matches_header():
    """INTEGRATION.md §2's ctypes binding: argtypes follow the header's
    ffddp_solve_batch signature and the stats buffer holds FFDDP_NSTATS words
    per instance (the library writes B * FFDDP_NSTATS int32)."""
    doc = (ROOT / "INTEGRATION.md").read_text()
    block = doc.split("## 2. ")[1].split("```python")[1].split("```")[0]
    hdr = HEADER.read_text()
    nstats = int(re.search(r"#define FFDDP_NSTATS (\d+)", hdr).group(1))
    assert nstats == _abi.NSTATS
    assert int(re.search(r"^FFDDP_NSTATS = (\d+)", block, re.M).group(1)) == nstats
    assert re.search(r"stats = np\.zeros\(\(1, FFDDP_NSTATS\), np\.int32\)", block)
    # argtypes vs the C prototype, parameter by parameter
    ns = {"C": ctypes, "D": ctypes.POINTER(ctypes.c_double), "I32": ctypes.POINTER(ctypes.c_int32),
          "U8": ctypes.POINTER(ctypes.c_uint8)}
    m = re.search(r"lib\.ffddp_solve_batch\.argtypes = (\[.*?\])", block, re.S)
    doc_types = eval(m.group(1), ns)  # noqa: S307 (our own documentation text)
    proto = re.search(r"int ffddp_solve_batch\((.*?)\);", hdr, re.S).group(1)
    cmap = {"ffddp_handle*": ctypes.c_void_p, "int": ctypes.c_int, "const double*": ns["D"], "double*": ns["D"],
            "const uint8_t*": ns["U8"], "uint8_t*": ns["U8"], "int32_t*": ns["I32"]}
    params = [" ".join(p.split()[:-1]).replace(" *", "*") for p in proto.replace("\n", " ").split(",")]
    assert [cmap[p] for p in params] == doc_types


def test_integration_plan_snippet_matches_header():
    """INTEGRATION.md's solve-plan binding: the PlanIO fields are
    ffddp_plan_io's, in order, and the create call's argtypes follow the
    prototype."""
    doc = (ROOT / "INTEGRATION.md").read_text()
    block = doc.split("### One graph launch per tick")[1].split("```python")[1].split("```")[0]
    hdr = HEADER.read_text()
    body = re.search(r"typedef struct ffddp_plan_io \{(.*?)\} ffddp_plan_io;", hdr, re.S).group(1)
    fields = re.findall(r"\*\s*(\w+);", body)
    doc_fields = re.findall(r'"(\w+)"', re.search(r"_fields_ = \[(.*?)\]\n", block, re.S).group(1))
    assert fields == doc_fields == [n for n, _ in _abi.PlanIO._fields_]
    proto = re.search(r"int ffddp_plan_create\((.*?)\);", hdr, re.S).group(1)
    assert len(proto.split(",")) == 6 and "lib.ffddp_plan_create.argtypes" in block
