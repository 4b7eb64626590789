"""casadi-free function descriptors: the casadi.Function surface CusadiFunction relies on
(CusadiFunction.py:28-95) and the artefact names the reference loads (mpc_controller_cusadi.py:28-34)."""
import os

import numpy as np
import pytest

from biped_pympc_amd import layout
from biped_pympc_amd.cusadi import CASADI_FUNCTION_DIR, Function, pdipm_function, qp_former_function


def test_reference_artefact_names_resolve():
    f = Function.load(os.path.join(CASADI_FUNCTION_DIR, "srbd_qp_mat.casadi"))
    s = Function.load(os.path.join(CASADI_FUNCTION_DIR,
                                   "mpc_multiple_iter_5_solver_240v_140eq_160ineq.casadi"))
    assert f.name() == "qp_former" and f.horizon == 10
    assert s.name() == "sparse_pdipm_multiple_iterations" and s.n_iter == 5
    s20 = Function.load(os.path.join(CASADI_FUNCTION_DIR, "mpc_multiple_iter_solver_240v_140eq_160ineq.casadi"))
    assert s20.n_iter == 20  # the CPU path's 20-iteration solver (mpc_controller_casadi.py:31)


@pytest.mark.parametrize("N", [10, 20])
def test_former_signature(N):
    f = qp_former_function(N)
    d = layout.Dims(N)
    assert f.n_in() == 17 and f.n_out() == 6
    assert [f.nnz_in(i) for i in range(17)] == list(d.former_in_nnz)
    assert [f.nnz_out(i) for i in range(6)] == list(d.former_out_nnz)
    assert (f.size1_out(2), f.size2_out(2)) == (d.n_eq, d.nz)
    assert (f.size1_in(12), f.size2_in(12)) == (N, 2)  # contact_table is N x 2 (srbd_constraints.py:50)
    rows, cols = f.sparsity_out(2).get_triplet()
    cp, ri = layout.ccs_A(N)
    assert rows == ri.tolist()
    assert cols == np.repeat(np.arange(d.nz), np.diff(cp)).tolist()


def test_solver_signature():
    s = pdipm_function(10, 5)
    assert s.n_in() == 10 and s.n_out() == 6
    assert [s.nnz_in(i) for i in range(10)] == [240, 280, 1196, 240, 160, 140, 240, 160, 160, 140]
    assert [s.nnz_out(i) for i in range(6)] == [240, 160, 160, 140, 4, 1]
    assert s.sz_w() == 0
    with pytest.raises(NotImplementedError):
        s.call([])


def test_descriptor_roundtrip(tmp_path):
    s = pdipm_function(20, 10)
    p = tmp_path / "x.json"
    s.save(str(p))
    t = Function.load(str(p))
    assert (t.name(), t.horizon, t.n_iter) == (s.name(), 20, 10)
    assert t.name() == "sparse_pdipm_multiple_iterations_N20_K10"


def test_bad_descriptors():
    with pytest.raises(ValueError):
        Function("pdipm", 10, 0)
    with pytest.raises(ValueError):
        Function("qp_former", 64)
    with pytest.raises(FileNotFoundError):
        Function.load("/nonexistent/thing.casadi")
