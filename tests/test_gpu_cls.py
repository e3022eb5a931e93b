"""GPU: the BPF front end (groundSeg::ground_seg + nongroundExtract::featureExtract,
include/preProcess.hpp:398-505 / :646-689, chained as src/additionNode.cpp:21-45) through the C ABI
(pf_cls_*) against the oracle.

Integer / index work, so the bar is bit-exact: the ground and non-ground push order, the radius
k-NN neighbour counts, every point's pillar / beam / facade decision and the order of the published
clouds equal the oracle's (both compute the PCA with the same f32 sums and f64 eigensolver)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def fe(pa):
    return pa.BPFFrontEnd(max_points=300000, device=0)


def _same(got, want):
    for k in ("beam", "pillar", "facade", "ground"):
        np.testing.assert_array_equal(got[k], want[k], err_msg=k)


@pytest.mark.parametrize("preset,frame", [("S64", 0), ("S64", 7), ("S32", 3)])
def test_extract_matches_oracle(pa, pfref, pfsynth, fe, preset, frame):
    x = pfsynth.Sequence(preset, n_frames=frame + 1).frame(frame)
    got = fe.extract(x)
    want = pfref.bpf_preprocess(x, pfref.cls_params())
    _same(got, want)
    assert len(got["facade"]) > 1000 and len(got["pillar"]) > 50 and len(got["ground"]) > 10000
    g, u = fe.ground_seg(x)                                     # pf_cls_ground_seg alone
    og, ou = pfref.ground_seg(x, pfref.cls_params())
    np.testing.assert_array_equal(g, og)
    np.testing.assert_array_equal(u, ou)


def test_classify_matches_oracle(pa, pfref, pfsynth, fe):
    x = pfsynth.Sequence("S64", n_frames=3).frame(2)
    g, u = pfref.ground_seg(x, pfref.cls_params())
    U = x[u]
    cls, num = fe.classify(U)
    ocls, onum = pfref.pca_classify(U, pfref.cls_params())
    np.testing.assert_array_equal(num, onum)
    np.testing.assert_array_equal(cls, ocls)
    assert np.all(num <= 25) and np.mean(num == 25) > 0.5


def test_normals_match_oracle(pa, pfref, pfsynth, fe):
    """pf_cls_normals: the normal assign_normal leaves in every point, bit-exact against the oracle
    (same f32 PCA sums, same f64 eigensolver rounded to f32): the class's direction for classified
    points, the PCA normal for other points with more than 3 neighbours (:238-239), zeros with 0-3."""
    x = pfsynth.Sequence("S64", n_frames=6).frame(5)
    g, u = pfref.ground_seg(x, pfref.cls_params())
    U = x[u]
    cls, num, nrm = fe.classify(U, normals=True)
    ocls, onum, onrm = pfref.pca_classify(U, pfref.cls_params(), normals=True)
    np.testing.assert_array_equal(cls, ocls)
    np.testing.assert_array_equal(nrm.view(np.uint32), onrm.view(np.uint32))
    on = num > 3
    np.testing.assert_allclose(np.linalg.norm(nrm[on, :3], axis=1), 1.0, atol=1e-5)
    assert np.all(nrm[~on] == 0)
    assert ((cls == 0) & on).sum() > 100                     # unclassified points with a normal


@pytest.mark.parametrize("kw", [dict(k=5), dict(k=32, k_min=3), dict(radius=0.5), dict(ground_filter=0),
                                dict(gf_grid_res=1.0, gf_min_grid_pts=3), dict(beam_h_min=-10.0, edge_thre=0.5)])
def test_parameters(pa, pfref, pfsynth, kw):
    x = pfsynth.Sequence("S32", n_frames=2, az_steps=900).frame(1)
    f = pa.BPFFrontEnd(max_points=200000, device=0, **kw)
    _same(f.extract(x), pfref.bpf_preprocess(x, pfref.cls_params(**kw)))


def test_edge_cases(pa, pfref, fe):
    rng = np.random.default_rng(11)
    cases = [np.zeros((0, 4), np.float32),                                   # empty scan
             np.array([[1, 2, 0, 0]], np.float32),                             # one point
             rng.uniform(-1, 1, (7, 4)).astype(np.float32),                    # fewer than one cell's minimum
             np.c_[rng.uniform(-5, 5, (500, 2)), rng.uniform(6, 9, 500), np.zeros(500)].astype(np.float32),  # all high
             np.repeat(np.array([[3.0, 4.0, -1.0, 0]], np.float32), 40, 0),   # duplicates: d^2 ties, x range 0
             np.c_[np.linspace(0, 2.9999, 300), np.linspace(0, 6, 300), np.full(300, -1.7), np.zeros(300)].astype(np.float32)]
    for x in cases:
        _same(fe.extract(x), pfref.bpf_preprocess(x, pfref.cls_params()))


def test_rejects(pa, pfsynth):
    with pytest.raises(pa.PFError):
        pa.BPFFrontEnd(max_points=1000, k=33)
    with pytest.raises(pa.PFError):
        pa.BPFFrontEnd(max_points=1000, radius=1.5)
    small = pa.BPFFrontEnd(max_points=1000)
    x = pfsynth.Sequence("S32", n_frames=1, az_steps=300).frame(0)
    with pytest.raises(pa.PFError):
        small.extract(x)                                                       # larger than max_points
    far = np.array([[0, 0, 0], [2000.0, 2000.0, 0]], np.float32)               # ground grid > 32766 cells
    with pytest.raises(pa.PFError):
        small.extract(far)


def test_matches_committed_fixture(pa, pfsynth, fe):
    """tests/golden/cls_s32_f2.npz (oracle output, tools/make_golden.py) reproduced on the device."""
    import hashlib
    import os
    g = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "cls_s32_f2.npz"))
    x = pfsynth.Sequence("S32", n_frames=3, az_steps=900).frame(2)
    assert hashlib.sha256(np.ascontiguousarray(x).tobytes()).hexdigest() == str(g["input_sha"])
    _same(fe.extract(x), {k: g[k] for k in ("beam", "pillar", "facade", "ground")})
    cls, num = fe.classify(x[g["unground"]])
    np.testing.assert_array_equal(cls, g["cls"])
    np.testing.assert_array_equal(num, g["pt_num"])


def _boundary_clouds(rng):
    """Clouds that put the search's index math at its edges: points exactly on 1 m cell faces (the
    query's cell at the grid's first / last x, y, z index, rows missing at the borders), a one-cell
    grid, axis lines on integer coordinates, chunks cut by cell ends (sizes around multiples of 16)
    and dense duplicates (d^2 ties)."""
    out = []
    for n in (1, 2, 15, 16, 17, 31, 33, 64, 65, 257, 1000, 4099):
        out.append(rng.integers(-2, 3, (n, 3)).astype(np.float32))             # integer lattice: all on faces
        out.append(rng.uniform(0.0, 0.999, (n, 3)).astype(np.float32))         # one cell
    t = np.linspace(-3, 3, 601, dtype=np.float32)
    z = np.zeros_like(t)
    out.append(np.c_[t, z, z])                                                  # line along x through cell faces
    out.append(np.c_[z, t, z + 1])                                              # along y
    out.append(np.c_[z + 2, z - 1, t])                                          # along z
    out.append(np.repeat(rng.uniform(-1, 1, (8, 3)), 40, 0).astype(np.float32))  # 8 points x 40 duplicates
    g = np.stack(np.meshgrid(*[np.arange(-1.5, 1.51, 0.25)] * 3), -1).reshape(-1, 3).astype(np.float32)
    out.append(g)                                                               # 13^3 grid, 0.25 m pitch
    out.append(np.r_[g, g + np.float32(0.5)])
    return out


def test_search_index_edges_match_oracle(pa, pfref, fe):
    """The radius k-NN search and PCA decision (k_cls_search / k_cls_decide) on clouds that stress
    the cell-row, chunk and border index math, bit-exact against the oracle, k = 25 and k = 32."""
    rng = np.random.default_rng(2024)
    f32 = pa.BPFFrontEnd(max_points=300000, device=0, k=32, k_min=3)
    for i, U in enumerate(_boundary_clouds(rng)):
        for f, prm in ((fe, pfref.cls_params()), (f32, pfref.cls_params(k=32, k_min=3))):
            cls, num = f.classify(U)
            ocls, onum = pfref.pca_classify(U, prm)
            np.testing.assert_array_equal(num, onum, err_msg="cloud %d (n=%d)" % (i, len(U)))
            np.testing.assert_array_equal(cls, ocls, err_msg="cloud %d (n=%d)" % (i, len(U)))
