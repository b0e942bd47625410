"""CPU tests of the oracle: the C restatement (maxk_oracle.c, main_inputs.cpp)
against the independent numpy restatement, the warp4 schedule semantics of
kernels/generate_meta.py:26-48, and main.cu's input generator."""
import numpy as np
import pytest

from spgemm_new_amd.graphs import random_cbsr, small_csr


@pytest.fixture(scope="module")
def graph():
    indptr, indices = small_csr(1200, seed=11)
    rng = np.random.default_rng(0)
    values = rng.random(len(indices), dtype=np.float32)
    return indptr, indices, values


def test_warp4_matches_generate_meta_semantics(oracle, graph):
    indptr, _, _ = graph
    w_c = oracle.c_warp4(indptr, 64)
    w_np = oracle.np_warp4(indptr, 64)
    np.testing.assert_array_equal(w_c, w_np)
    deg = np.diff(indptr)
    # degree-0 rows produce no chunk (generate_meta.py:32-33)
    assert set(np.unique(w_c[:, 0])) == set(np.nonzero(deg)[0])
    # chunks tile the edge range contiguously, <= 64 each
    assert np.all(w_c[:, 2] <= 64) and np.all(w_c[:, 2] >= 1)
    assert w_c[0, 1] == 0
    np.testing.assert_array_equal(w_c[1:, 1], w_c[:-1, 1] + w_c[:-1, 2])
    assert w_c[-1, 1] + w_c[-1, 2] == indptr[-1]
    # a 65-edge row is split 64 + 1 (generate_meta.py:36-45)
    r65 = int(np.nonzero(deg == 65)[0][0])
    ch = w_c[w_c[:, 0] == r65]
    assert ch[:, 2].tolist() == [64, 1]


@pytest.mark.parametrize("k", [4, 8, 16, 32, 64, 5])
@pytest.mark.parametrize("h", [256, 64])
def test_forward_c_vs_numpy(oracle, graph, k, h):
    indptr, indices, values = graph
    if k > h:
        pytest.skip("k > h")
    data, sel = random_cbsr(len(indptr) - 1, k, h, seed=k)
    w4 = oracle.c_warp4(indptr)
    y_c = oracle.c_forward(w4, indices, values, data, sel, h)
    y_np = oracle.np_forward(indptr, indices, values, data, sel, h)
    assert oracle.parity_error(y_c, y_np) < 1e-5
    y_csr = oracle.c_forward_csr(indptr, indices, values, data, sel, h)
    assert oracle.parity_error(y_csr, y_np) < 1e-5


@pytest.mark.parametrize("k", [4, 8, 16, 32, 64, 5])
def test_backward_c_vs_numpy(oracle, graph, k):
    indptr, indices, values = graph
    h = 256
    v = len(indptr) - 1
    _, sel = random_cbsr(v, k, h, seed=100 + k)
    grad = np.random.default_rng(k).random((v, h), dtype=np.float32)
    w4 = oracle.c_warp4(indptr)
    d_c = oracle.c_backward(w4, indices, values, grad, sel)
    d_np = oracle.np_backward(indptr, indices, values, grad, sel)
    assert oracle.parity_error(d_c, d_np) < 1e-5
    d_csr = oracle.c_backward_csr(indptr, indices, values, grad, sel)
    assert oracle.parity_error(d_csr, d_np) < 1e-5


def test_backward_is_adjoint_of_forward(oracle, graph):
    """<A.scatter(Xs), G> == <Xs, (A^T G)|sel> for every CBSR pair (exact adjoint)."""
    indptr, indices, values = graph
    v, h, k = len(indptr) - 1, 256, 16
    data, sel = random_cbsr(v, k, h, seed=3)
    grad = np.random.default_rng(5).random((v, h))
    y = oracle.np_forward(indptr, indices, values, data, sel, h)
    dxs = oracle.np_backward(indptr, indices, values, grad, sel)
    lhs = float(np.sum(y * grad))
    rhs = float(np.sum(data.astype(np.float64) * dxs))
    assert abs(lhs - rhs) <= 1e-9 * abs(lhs)


def test_main_inputs_generator(oracle):
    """main.cu:74-146: deterministic, distinct selectors in [0,256), U(0,1) values,
    and the k=32 stream depends on the k=16 draws before it (same engine)."""
    v, e = 50, 400
    a = oracle.c_main_inputs(v, e, 32, densify=True)
    b = oracle.c_main_inputs(v, e, 32, densify=True)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)
    values, data, sel, dense = a
    assert values.shape == (e,) and np.all((values >= 0) & (values < 1))
    assert data.shape == (v, 32) and np.all((data >= 0) & (data < 1))
    for r in range(v):
        assert len(set(sel[r].tolist())) == 32
        # std::sample keeps the relative order of the population (ascending)
        assert np.all(np.diff(sel[r].astype(int)) > 0)
    np.testing.assert_array_equal(np.count_nonzero(dense, axis=1), 32)
    v16 = oracle.c_main_inputs(v, e, 16)
    np.testing.assert_array_equal(v16[0], values)           # same edge values
    assert not np.array_equal(v16[2][:, :16], sel[:, :16])  # k=32 drawn after k=16


def test_c_backward_rectangular_block(oracle):
    """The C restatements size dXs by A's columns: a row block with halo
    columns (num_cols > num_rows) agrees with the numpy oracle."""
    from spgemm_new_amd.graphs import random_cbsr
    rng = np.random.default_rng(3)
    rows, cols, h, k = 150, 420, 64, 8
    deg = rng.integers(0, 30, rows)
    indptr = np.zeros(rows + 1, np.int32)
    indptr[1:] = np.cumsum(deg)
    indices = np.concatenate([np.sort(rng.choice(cols, d, replace=False)) for d in deg]).astype(np.int32)
    values = rng.random(indices.size, dtype=np.float32)
    _, sel = random_cbsr(cols, k, h, seed=4)
    grad = rng.random((rows, h), dtype=np.float32)
    ref = oracle.np_backward(indptr, indices, values, grad, sel)
    assert ref.shape == (cols, k)
    got = oracle.c_backward_csr(indptr, indices, values, grad, sel)
    assert got.shape == (cols, k) and oracle.parity_error(got, ref) <= 1e-5
    w4 = oracle.c_warp4(indptr)
    got4 = oracle.c_backward(w4, indices, values, grad, sel)
    assert got4.shape == (cols, k) and oracle.parity_error(got4, ref) <= 1e-5
