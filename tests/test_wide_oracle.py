"""CPU checks of the oracle's wide-path contraction (NP8O_CONTRACT_F32, DESIGN.md "Wide path").

The oracle restates the fp32 MFMA contraction (fmaf chains over 16-row tiles) that np8_assign_wide
runs on the device; tests/test_gpu_wide.py pins device = oracle bit for bit.  Here the oracle's fp32
likelihoods are checked against its fp64 formula with the general inverse
(multivariatenormal.cpp:106-136) at tiled and padded D (20, 40, 80 are not multiples of 16), within the tolerance the GPU tests use, and the
oracle's wide sweeps are checked to keep the membertrix invariants.
"""
import numpy as np
import pytest

import oracle as O

F32_LL_RTOL = 1e-5  # as tests/test_gpu_wide.py


def mixture(D, N, K, seed, spread=5.0):
    rng = np.random.default_rng(seed)
    cent = rng.uniform(-spread, spread, size=(K, D))
    z = rng.integers(0, K, N)
    return cent[z] + rng.normal(size=(N, D)), z, cent


def chain(D, prior, seed):
    if prior == "niw":
        kw = dict(mu0=np.zeros(D), kappa=0.05, nu=D + 2.0, Lambda=0.5 * np.eye(D), prior="niw")
    else:
        kw = dict(mu0=np.zeros(D), kappa=0.02, nu=4.0, Lambda=np.eye(D) / D**2)
    return O.Chain(D, contraction="f32", kcap=256, seed=seed, **kw)


@pytest.mark.parametrize("D", [20, 32, 40, 48, 64, 80])
@pytest.mark.parametrize("prior", ["reference", "niw"])
def test_wide_contraction_against_fp64_formula(D, prior):
    X, _, _ = mixture(D, 600, 6, D)
    o = chain(D, prior, 3)
    o.set_data(X)
    o.init_random(8)
    idx = np.arange(0, 600, 13)
    lw, ref = o.loglik_matrix(idx), o.loglik_matrix(idx, ref=True)
    K = o.K
    np.testing.assert_allclose(lw[:, :K], ref[:, :K], rtol=F32_LL_RTOL)


@pytest.mark.parametrize("D", [48])
def test_wide_sweeps_keep_invariants(D):
    X, z, cent = mixture(D, 800, 5, 7 + D)
    o = chain(D, "reference", 11)
    o.set_data(X)
    o.set_state(z.astype(np.int32), cent, np.repeat(np.eye(D)[None], 5, axis=0))
    for _ in range(3):
        o.sweep(1)
        s = o.state()
        assert s["counts"].sum() == 800
        assert (s["counts"][: s["K"]] > 0).all()
        assert s["z"].min() >= 0 and s["z"].max() < s["K"]


@pytest.mark.parametrize("D", [16, 81])
def test_wide_rejects_dimension_outside_range(D):
    """The wide path covers 16 < D <= 80 (any D: the device pads to the next multiple of 16); D <= 16 is the fp64
    path's."""
    with pytest.raises(Exception):
        O.Chain(D, contraction="f32", kcap=256, mu0=np.zeros(D), kappa=0.02, nu=4.0, Lambda=np.eye(D))
