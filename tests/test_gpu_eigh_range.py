"""GPU check of tg_eigh_vectors_range for a few dropped eigenpairs (the
complement path's request: count ~ 1-50 starting at k), on the two-stage
eigensolver, including a range ending at the last eigenvector.

Bars (as tests/test_gpu_solver.py::test_eigh): residual ||H v - lambda v|| <=
1e-10 ||H||, orthogonality <= 1e-10, and agreement with LAPACK's eigenvectors
up to sign where the eigenvalue gap is large.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _wishart(n, seed):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((3 * n // 2, n))
    return X.T @ X / X.shape[0]


def _blockdiag(n, seed):
    """Wishart block + a diagonal tail: the tridiagonal splits into an
    unreduced block and 1x1 blocks (exercises the block-local solves)."""
    nb = n // 2
    H = np.zeros((n, n))
    H[:nb, :nb] = _wishart(nb, seed)
    H[nb:, nb:] = np.diag(np.linspace(0.05, 2.5, n - nb))
    return H


# count <= 256: one LDS-resident wave per vector (invit_lds_kernel);
# count > 256: the register path (invit_kernel)
@pytest.mark.parametrize("n,first,count,kind", [
    (600, 0, 14, "wishart"), (2048, 1500, 14, "wishart"), (2048, 0, 48, "wishart"),
    (4100, 3058, 14, "wishart"), (4100, 4099, 1, "wishart"), (1000, 0, 300, "wishart"),
    (6000, 4500, 14, "wishart"),
    (700, 0, 20, "blockdiag"), (700, 640, 60, "blockdiag")])
def test_few_vectors(n, first, count, kind):
    from gptq_svd_amd import _lib as lib
    H = _wishart(n, n + first) if kind == "wishart" else _blockdiag(n, n + first)
    A = torch.from_numpy(H).to(DEV)
    ws = lib.workspace(lib.lib.tg_eigh_workspace_size(n), torch.device(DEV))
    w = torch.empty(n, dtype=torch.float64, device=DEV)
    lib.call("tg_eigh_values", lib.stream(), lib.ptr(A), n, n, lib.ptr(w), lib.ptr(ws), ws.numel())
    V = torch.empty((count, n), dtype=torch.float64, device=DEV)
    lib.call("tg_eigh_vectors_range", lib.stream(), n, lib.ptr(w), first, count, lib.ptr(V), n,
             lib.ptr(ws), ws.numel())
    torch.cuda.synchronize()
    Vh = V.cpu().numpy()
    lam_desc = w.cpu().numpy()[::-1]
    lam = lam_desc[first:first + count]
    nrm = np.abs(lam_desc).max()
    resid = np.linalg.norm(Vh @ H - lam[:, None] * Vh, axis=1).max()
    assert resid <= 1e-10 * nrm, resid
    orth = np.abs(Vh @ Vh.T - np.eye(count)).max()
    assert orth <= 1e-10, orth
    L, Q = np.linalg.eigh(H)
    Qd = Q[:, ::-1][:, first:first + count].T
    gaps = np.abs(np.diff(L[::-1]))
    for j in range(count):
        g = min(gaps[first + j - 1] if first + j > 0 else np.inf,
                gaps[first + j] if first + j < n - 1 else np.inf)
        if g > 1e-6 * nrm:
            assert abs(abs(Vh[j] @ Qd[j]) - 1.0) <= 1e-8


def _spectrum(n, kind, seed):
    rng = np.random.default_rng(seed)
    Q = np.linalg.qr(rng.standard_normal((n, n)))[0]
    if kind == "graded":        # 1e-10 .. 1: the bottom ~60% forms one ortol cluster
        lam = np.logspace(-10, 0, n)
    elif kind == "clustered":   # four 64-fold near-multiple eigenvalues + a dense rest
        lam = np.linspace(0.1, 1.0, n)
        for c, v in enumerate((0.2, 0.45, 0.7, 0.95)):
            lam[c * 64:(c + 1) * 64] = v * (1 + 1e-12 * rng.standard_normal(64))
        lam.sort()
    else:
        raise ValueError(kind)
    return (Q * lam) @ Q.T


@pytest.mark.parametrize("kind,first,count", [("graded", 0, 4096), ("clustered", 0, 4096),
                                              ("graded", 1200, 600), ("clustered", 3000, 400)])
def test_orthogonality_n4096(kind, first, count):
    """Eigenvectors at n = 4096 with graded / clustered spectra: inverse
    iteration + cluster re-orthogonalisation (ortol 1e-6 ||T||, block
    Gram-Schmidt for big clusters) keeps them orthogonal to <= 1e-9."""
    from gptq_svd_amd import _lib as lib
    n = 4096
    H = _spectrum(n, kind, 11 + first)
    A = torch.from_numpy(H).to(DEV)
    Hd = A.clone()
    ws = lib.workspace(lib.lib.tg_eigh_workspace_size(n), torch.device(DEV))
    w = torch.empty(n, dtype=torch.float64, device=DEV)
    lib.call("tg_eigh_values", lib.stream(), lib.ptr(A), n, n, lib.ptr(w), lib.ptr(ws), ws.numel())
    V = torch.empty((count, n), dtype=torch.float64, device=DEV)
    lib.call("tg_eigh_vectors_range", lib.stream(), n, lib.ptr(w), first, count, lib.ptr(V), n,
             lib.ptr(ws), ws.numel())
    lam = torch.flip(w, [0])[first:first + count]
    nrm = float(w.abs().max())
    resid = float(torch.linalg.norm(V @ Hd - lam[:, None] * V, dim=1).max())
    orth = float((V @ V.T - torch.eye(count, dtype=torch.float64, device=DEV)).abs().max())
    print(f"{kind} n={n} [{first}, {first + count}): resid {resid / nrm:.2e} ||H||, orth {orth:.2e}")
    assert resid <= 1e-10 * nrm
    assert orth <= 1e-9


def test_panel_pairs_large_n(monkeypatch):
    """n = 9000: the default band reduction pairs the panels with >= 6144
    trailing rows (merged rank-128 updates, corrections on a side stream);
    its eigenvalues match the unpaired reduction's (TG_SB_PAIR=0) to
    1e-12 ||H|| and repeat bit for bit."""
    from gptq_svd_amd import _lib as lib
    n = 9000
    H = torch.from_numpy(_wishart(n, 4)).to(DEV)
    ws = lib.workspace(lib.lib.tg_eigh_workspace_size(n), torch.device(DEV))

    def values(pair):
        if pair is None:
            monkeypatch.delenv("TG_SB_PAIR", raising=False)
        else:
            monkeypatch.setenv("TG_SB_PAIR", pair)
        A = H.clone()
        w = torch.empty(n, dtype=torch.float64, device=DEV)
        lib.call("tg_eigh_values", lib.stream(), lib.ptr(A), n, n, lib.ptr(w), lib.ptr(ws),
                 ws.numel())
        torch.cuda.synchronize()
        return w.cpu().numpy()

    paired, plain = values(None), values("0")
    assert np.array_equal(values(None), paired)
    nrm = np.abs(plain).max()
    assert np.abs(paired - plain).max() <= 1e-12 * nrm


@pytest.mark.parametrize("n,count", [(4096, 14), (2048, 32)])
def test_q2_wavefront_bit_identical(n, count, monkeypatch):
    """The few-vector back-transform's Q2 part as a wavefront of sweep
    groups (point-to-point progress words, TG_BT_Q2_WAVE=1) gives the level-by-
    level form's eigenvectors bit for bit (same blocks, same arithmetic,
    same order on every row), twice in a row."""
    from gptq_svd_amd import _lib as lib
    H = torch.from_numpy(_wishart(n, 9)).to(DEV)
    ws = lib.workspace(lib.lib.tg_eigh_workspace_size(n), torch.device(DEV))

    def vectors(wave):
        monkeypatch.setenv("TG_BT_Q2_WAVE", wave)
        A = H.clone()
        w = torch.empty(n, dtype=torch.float64, device=DEV)
        lib.call("tg_eigh_values", lib.stream(), lib.ptr(A), n, n, lib.ptr(w), lib.ptr(ws),
                 ws.numel())
        V = torch.empty((count, n), dtype=torch.float64, device=DEV)
        lib.call("tg_eigh_vectors_range", lib.stream(), n, lib.ptr(w), n - count, count,
                 lib.ptr(V), n, lib.ptr(ws), ws.numel())
        torch.cuda.synchronize()
        return V.cpu().numpy()

    ref = vectors("0")
    for _ in range(2):
        assert np.array_equal(vectors("1"), ref)


@pytest.mark.parametrize("n", [6400, 9000])
def test_xm_asm_loads_bit_identical(n, monkeypatch):
    """The X/M kernel's hand-written K loop (inline-asm loads with counted
    waits, csrc/band.hip xm_load_asm, the default) against the compiler-
    scheduled loop (TG_XM_ASM=0) on the paired path (trailing matrices of
    >= 6144 rows: xm_kernel<2> with the pair products): the same MFMAs in the
    same order, so the reduced matrix left in A and the eigenvalues must agree
    bit for bit.  A register read before its load landed would show here;
    tools/check_xm_isa.py guards the same loop statically in build()."""
    from gptq_svd_amd import _lib as lib
    H = torch.from_numpy(_wishart(n, 12)).to(DEV)
    ws = lib.workspace(lib.lib.tg_eigh_workspace_size(n), torch.device(DEV))

    def values(asm):
        if asm is None:
            monkeypatch.delenv("TG_XM_ASM", raising=False)
        else:
            monkeypatch.setenv("TG_XM_ASM", asm)
        A = H.clone()
        w = torch.empty(n, dtype=torch.float64, device=DEV)
        lib.call("tg_eigh_values", lib.stream(), lib.ptr(A), n, n, lib.ptr(w), lib.ptr(ws),
                 ws.numel())
        torch.cuda.synchronize()
        return w.cpu().numpy(), A

    w_asm, A_asm = values(None)
    w_cc, A_cc = values("0")
    assert torch.equal(A_asm, A_cc)
    assert np.array_equal(w_asm, w_cc)


@pytest.mark.parametrize("n,switches", [
    (1025, {"TG_XM_NBC": "2"}), (1025, {"TG_XM_NBC": "2", "TG_XM_ASM": "0"}),
    (1999, {"TG_XM_NBC": "2"}), (6401, {})])
def test_xm_packed_odd_width(n, switches, monkeypatch):
    """the packed X/M loads (NBC = 2, two adjacent A22 columns per
    16-byte load) at an odd trailing width m: the pair (m - 1, m) is loaded
    one column left and column m - 1 must take the load's second element.
    Every panel's m has n's parity, so an odd n runs the tail pair on every
    panel (n = 6401 takes NBC = 2 by default).  Eigenvalues vs LAPACK to
    1e-12 ||H|| and vs the unpacked NBC = 1 kernel to 1e-12 ||H||."""
    from gptq_svd_amd import _lib as lib
    H = _wishart(n, 31)
    ws = lib.workspace(lib.lib.tg_eigh_workspace_size(n), torch.device(DEV))

    def values(env):
        for k in ("TG_XM_NBC", "TG_XM_ASM"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        A = torch.from_numpy(H).to(DEV)
        w = torch.empty(n, dtype=torch.float64, device=DEV)
        lib.call("tg_eigh_values", lib.stream(), lib.ptr(A), n, n, lib.ptr(w), lib.ptr(ws),
                 ws.numel())
        torch.cuda.synchronize()
        return np.sort(w.cpu().numpy())

    got = values(switches)
    nrm = np.abs(got).max()
    ref = np.linalg.eigvalsh(H)
    assert np.abs(got - ref).max() <= 1e-12 * nrm, np.abs(got - ref).max() / nrm
    one = values({"TG_XM_NBC": "1"})
    assert np.abs(got - one).max() <= 1e-12 * nrm


@pytest.mark.parametrize("n,count", [(4096, 14), (4096, 16), (1000, 1), (600, 14), (4100, 14),
                                     (9000, 14)])
def test_q2_lds_bit_identical(n, count, monkeypatch):
    """The few-vector Q2 with Z resident in LDS (csrc/backtr.hip
    q2_lds_kernel, the default for <= 16 vectors: one wave per pair column
    of blocks, LDS progress counters inside a workgroup, write-through
    boundary chunks between workgroups) gives the level-by-level form's
    eigenvectors (TG_BT_Q2_LDS=0) bit for bit, twice in a row -- partial last
    workgroups (n = 600, 1000), n not a multiple of 32, and more workgroups
    than one XCD has CUs (n = 9000: 36)."""
    from gptq_svd_amd import _lib as lib
    H = torch.from_numpy(_wishart(n, 17)).to(DEV)
    ws = lib.workspace(lib.lib.tg_eigh_workspace_size(n), torch.device(DEV))

    def vectors(flag):
        monkeypatch.setenv("TG_BT_Q2_LDS", flag)
        A = H.clone()
        w = torch.empty(n, dtype=torch.float64, device=DEV)
        lib.call("tg_eigh_values", lib.stream(), lib.ptr(A), n, n, lib.ptr(w), lib.ptr(ws),
                 ws.numel())
        V = torch.empty((count, n), dtype=torch.float64, device=DEV)
        lib.call("tg_eigh_vectors_range", lib.stream(), n, lib.ptr(w), n - count, count,
                 lib.ptr(V), n, lib.ptr(ws), ws.numel())
        torch.cuda.synchronize()
        return V.cpu().numpy()

    ref = vectors("0")
    for _ in range(2):
        assert np.array_equal(vectors("1"), ref)


@pytest.mark.parametrize("n,count", [(4096, 14), (4096, 1), (600, 14), (1000, 16), (3000, 14),
                                     (4000, 14), (4200, 14), (9000, 14)])
def test_q1_lds_bit_identical(n, count, monkeypatch):
    """The few-vector Q1 with Z resident in LDS (csrc/backtr.hip
    q1_lds_kernel, the default after q2_lds_kernel on single-level plans up
    to n = 4096: one 128-row sub-chunk of Z per workgroup, the workgroups of
    one XCD, one exchange of sub-chunk partials per panel step) gives
    bt_few_kernel's Q1 (TG_BT_Q1_LDS=0) bit for bit, twice in a row: both
    form the same row-aligned sub-chunk partials, sum them in the same order
    and form M = T P with the same MFMA sequence.  TG_BT_Q1_LDS=2 launches
    too few workgroups for one XCD, so the election fails and bt_few's Q1
    runs instead: the same vectors again.  n = 3000 / 4000 / 600: a partial
    last sub-chunk; n = 4096: all 32 CUs of the XCD; n = 4200 / 9000: 33 / 71
    sub-chunks, more than one XCD's CUs: the placement-independent form
    (q1_lds_kernel<false>, write-through partials, one workgroup per CU)."""
    from gptq_svd_amd import _lib as lib
    H = torch.from_numpy(_wishart(n, 23)).to(DEV)
    ws = lib.workspace(lib.lib.tg_eigh_workspace_size(n), torch.device(DEV))

    def vectors(flag):
        monkeypatch.setenv("TG_BT_Q1_LDS", flag)
        A = H.clone()
        w = torch.empty(n, dtype=torch.float64, device=DEV)
        lib.call("tg_eigh_values", lib.stream(), lib.ptr(A), n, n, lib.ptr(w), lib.ptr(ws),
                 ws.numel())
        V = torch.empty((count, n), dtype=torch.float64, device=DEV)
        lib.call("tg_eigh_vectors_range", lib.stream(), n, lib.ptr(w), n - count, count,
                 lib.ptr(V), n, lib.ptr(ws), ws.numel())
        torch.cuda.synchronize()
        return V.cpu().numpy()

    ref = vectors("0")
    for _ in range(2):
        assert np.array_equal(vectors("1"), ref)
    assert np.array_equal(vectors("2"), ref)


@pytest.mark.parametrize("n,count,kind,iters", [(4096, 14, "wishart", "2"), (600, 14, "wishart", "3"),
                                                (700, 60, "blockdiag", "2"), (2048, 1, "wishart", "1")])
def test_invit_factor_once_bit_identical(n, count, kind, iters, monkeypatch):
    """Inverse iteration (csrc/eigh.hip invit_lds_kernel) factors T - lambda I
    once and keeps the multipliers (in the vector's Z column) and the row
    interchanges (LDS bit masks), so the later iterations only substitute:
    the vectors equal those of a kernel that factors in every iteration
    (TG_INVIT_REFACTOR=1) bit for bit -- 1, 2 and 3 iterations, and a
    block-diagonal T (1x1 blocks: m = 1, no forward step)."""
    from gptq_svd_amd import _lib as lib
    H = _wishart(n, 31) if kind == "wishart" else _blockdiag(n, 31)
    Hd = torch.from_numpy(H).to(DEV)
    ws = lib.workspace(lib.lib.tg_eigh_workspace_size(n), torch.device(DEV))
    monkeypatch.setenv("TG_INVIT_ITERS", iters)

    def vectors(refac):
        monkeypatch.setenv("TG_INVIT_REFACTOR", refac)
        A = Hd.clone()
        w = torch.empty(n, dtype=torch.float64, device=DEV)
        lib.call("tg_eigh_values", lib.stream(), lib.ptr(A), n, n, lib.ptr(w), lib.ptr(ws),
                 ws.numel())
        V = torch.empty((count, n), dtype=torch.float64, device=DEV)
        lib.call("tg_eigh_vectors_range", lib.stream(), n, lib.ptr(w), n - count, count,
                 lib.ptr(V), n, lib.ptr(ws), ws.numel())
        torch.cuda.synchronize()
        return V.cpu().numpy()

    ref = vectors("1")
    assert np.array_equal(vectors("0"), ref)


@pytest.mark.parametrize("n", [4096, 2000, 7000])
def test_xm_fused_w_bit_identical(n, monkeypatch):
    """W = X - Y M / 2 formed inside the X / M launch (csrc/band.hip
    xm_fused_w, TG_XM_FUSE_W=1: every workgroup waits for the last arriver's
    M, then updates its own rows; measured no faster, so opt-in) gives the
    reduced band of w_update_kernel (the default) bit for bit: the same fma
    chain per entry, so the eigenvalues agree exactly.  n = 2000: a ragged last row block; n = 7000: panels of both
    X / M forms (16 and 32 columns per workgroup) and panel pairs."""
    from gptq_svd_amd import _lib as lib
    H = torch.from_numpy(_wishart(n, 41)).to(DEV)
    ws = lib.workspace(lib.lib.tg_eigh_workspace_size(n), torch.device(DEV))

    def values(flag):
        monkeypatch.setenv("TG_XM_FUSE_W", flag)
        A = H.clone()
        w = torch.empty(n, dtype=torch.float64, device=DEV)
        lib.call("tg_eigh_values", lib.stream(), lib.ptr(A), n, n, lib.ptr(w), lib.ptr(ws),
                 ws.numel())
        torch.cuda.synchronize()
        return w.cpu().numpy()

    ref = values("0")
    for _ in range(2):
        assert np.array_equal(values("1"), ref)


@pytest.mark.parametrize("n,count", [(4096, 14), (3001, 5)])
def test_invit_global_rows_bit_identical(n, count, monkeypatch):
    """Inverse iteration with the rows in a per-vector global slab (csrc/
    eigh.hip invit_lds_kernel<true>, the default past n = 5120 where the
    rows do not fit the LDS; TG_INVIT_GROWS=1 forces it) gives the LDS-row
    kernel's vectors bit for bit (same operations; only where the rows live
    and how far ahead they are fetched differ)."""
    from gptq_svd_amd import _lib as lib
    H = torch.from_numpy(_wishart(n, 43)).to(DEV)
    ws = lib.workspace(lib.lib.tg_eigh_workspace_size(n), torch.device(DEV))

    def vectors(flag):
        monkeypatch.setenv("TG_INVIT_GROWS", flag)
        A = H.clone()
        w = torch.empty(n, dtype=torch.float64, device=DEV)
        lib.call("tg_eigh_values", lib.stream(), lib.ptr(A), n, n, lib.ptr(w), lib.ptr(ws),
                 ws.numel())
        V = torch.empty((count, n), dtype=torch.float64, device=DEV)
        lib.call("tg_eigh_vectors_range", lib.stream(), n, lib.ptr(w), n - count, count,
                 lib.ptr(V), n, lib.ptr(ws), ws.numel())
        torch.cuda.synchronize()
        return V.cpu().numpy()

    ref = vectors("0")
    assert np.array_equal(vectors("1"), ref)


@pytest.mark.parametrize("n", [4096, 2000, 7000, 9001])
def test_xm_ksplit(n, monkeypatch):
    """The X / M kernel with K split over several workgroups per column
    block (csrc/band.hip xm_ksplit: by default the 32-column form's grid is
    brought to ~1536 workgroups; TG_XM_KSPLIT=3 forces three splits of every
    launch; partial X blocks summed in split order by the last of a block's
    splits): eigenvalues equal LAPACK's and the unsplit kernel's
    (TG_XM_KSPLIT=1) to 1e-12 ||H||, and repeat bit for bit.  n = 7000 /
    9001: the 32-column form, panel pairs, an odd width; n = 2000 / 4096:
    the 16-column form (forced splits only)."""
    from gptq_svd_amd import _lib as lib
    H = _wishart(n, 47)
    ws = lib.workspace(lib.lib.tg_eigh_workspace_size(n), torch.device(DEV))

    def values(split):
        if split is None:
            monkeypatch.delenv("TG_XM_KSPLIT", raising=False)
        else:
            monkeypatch.setenv("TG_XM_KSPLIT", split)
        A = torch.from_numpy(H).to(DEV)
        w = torch.empty(n, dtype=torch.float64, device=DEV)
        lib.call("tg_eigh_values", lib.stream(), lib.ptr(A), n, n, lib.ptr(w), lib.ptr(ws),
                 ws.numel())
        torch.cuda.synchronize()
        return np.sort(w.cpu().numpy())

    got = values(None)
    assert np.array_equal(values(None), got)
    nrm = np.abs(got).max()
    ref = np.linalg.eigvalsh(H)
    assert np.abs(got - ref).max() <= 1e-12 * nrm
    forced = values("3")
    assert np.array_equal(values("3"), forced)
    assert np.abs(forced - ref).max() <= 1e-12 * nrm
    assert np.abs(got - values("1")).max() <= 1e-12 * nrm


@pytest.mark.parametrize("n,count", [(4096, 40), (3000, 24), (2048, 128), (9000, 43), (4100, 70)])
def test_few_slabs(n, count, monkeypatch):
    """Few-vector back-transform in 16-column slabs (csrc/backtr.hip
    sb_apply_few, k = 17 .. 128: q2_lds_kernel and q1_lds_kernel<false> with
    the slabs side by side in blockIdx.y, as many a launch as leave every
    workgroup a CU): the eigenpair bars of test_few_vectors, and every slab
    equals a call for its columns alone bit for bit (inverse iteration is per
    vector; each slab is the same arithmetic as a k <= 16 call).  Up to 32
    columns, also bt_few_kernel's vectors (TG_BT_SLABS=0) to 1e-12.  n = 2048,
    128: 8 slabs, Q1 in launches of 3; n = 9000, 43: a partial last slab,
    71 workgroups a slab; n = 4100: a ragged last sub-chunk."""
    from gptq_svd_amd import _lib as lib
    H = _wishart(n, 53)
    Hd = torch.from_numpy(H).to(DEV)
    ws = lib.workspace(lib.lib.tg_eigh_workspace_size(n), torch.device(DEV))
    A = Hd.clone()
    w = torch.empty(n, dtype=torch.float64, device=DEV)
    lib.call("tg_eigh_values", lib.stream(), lib.ptr(A), n, n, lib.ptr(w), lib.ptr(ws), ws.numel())
    first = n - count

    def vectors(f, c):
        V = torch.empty((c, n), dtype=torch.float64, device=DEV)
        lib.call("tg_eigh_vectors_range", lib.stream(), n, lib.ptr(w), f, c, lib.ptr(V), n,
                 lib.ptr(ws), ws.numel())
        torch.cuda.synchronize()
        return V.cpu().numpy()

    Vh = vectors(first, count)
    assert np.array_equal(vectors(first, count), Vh)
    lam_desc = w.cpu().numpy()[::-1]
    lam = lam_desc[first:]
    nrm = np.abs(lam_desc).max()
    resid = np.linalg.norm(Vh @ H - lam[:, None] * Vh, axis=1).max()
    assert resid <= 1e-10 * nrm, resid
    assert np.abs(Vh @ Vh.T - np.eye(count)).max() <= 1e-10
    for s in range(0, count, 16):
        c = min(16, count - s)
        assert np.array_equal(vectors(first + s, c), Vh[s:s + c]), s
    if count <= 32:
        monkeypatch.setenv("TG_BT_SLABS", "0")
        assert np.abs(vectors(first, count) - Vh).max() <= 1e-12
