"""CPU: the `--noise` plugin surface (idn.noise_spec) resolves spec strings to the recipes the
reference's dispatch produces (README.md:82-107; lib/model/test.py:1611-1831 for test_v0,
lib/roi_data_layer/minibatch.py:1518-1673 for train_v0)."""
import random

import pytest

from idn import noise_spec as ns


def ops(p):
    return [(s.kind, s.op) + tuple(s.args) for s in p.steps]


R = random.Random


# ---- canonical (README grammar) -----------------------------------------------------------
@pytest.mark.parametrize("spec,steps,out", [
    ("gaussian_var0.1", [("noise", "gaussian", 0.1), ("cast_u8", "u8")], "u8"),
    ("gaussian_median_var1.0", [("noise", "gaussian", 1.0), ("cast_u8", "u8"), ("filter", "median", 3)], "u8"),
    ("sap_mean_var0.8", [("noise", "sap", 0.8), ("cast_u8", "u8"), ("filter", "mean", 3)], "u8"),
    ("speckle_bilateral_var2.0", [("noise", "speckle", 2.0), ("cast_u8", "u8"),
                                  ("filter", "bilateral", 9, 20.0, 100.0)], "u8"),
    ("poisson", [("noise", "poisson"), ("cast_u8", "u8")], "u8"),
    ("poisson_wavelet", [("noise", "poisson"), ("cast_u8", "u8"), ("filter", "wavelet", "bior1.5", None)], "u8"),
    ("gaussian_wavelet_var1.5", [("noise", "gaussian", 1.5), ("filter", "wavelet", "bior1.5", None)], "u8"),
    ("periodic_gaus_blur_var100", [("noise", "periodic", 100.0), ("filter", "gaus_blur", 3)], "u8"),
    ("periodic_varsize", [("noise", "periodic", "size")], "u8"),
    ("original", [("noise", "original")], "u8"),
    ("original_median", [("noise", "original"), ("filter", "median", 3)], "u8"),
    ("bloom", [("noise", "bloom")], "u8"),
    ("shader", [("noise", "shader")], "u8"),
])
def test_canonical(spec, steps, out):
    p = ns.plan(spec, "canonical", R(0))
    assert ops(p) == steps and p.out_dtype == out


def test_canonical_mix_inserts_denoiser():
    seen = set()
    for s in range(200):
        p = ns.plan("noise_mix_var_low_median", "canonical", R(s))
        assert p.spec == "noise_mix_var_low_median"
        seen.add(p.steps[0].op)
        if p.steps[0].op in ("gaussian", "sap", "speckle", "poisson"):
            assert p.steps[-1].op == "median"
    assert {"gaussian", "poisson", "speckle", "sap", "periodic", "original"} <= seen


def test_canonical_rejects_unknown():
    with pytest.raises(ValueError):
        ns.plan("fog_var0.1", "canonical", R(0))
    with pytest.raises(ValueError):
        ns.plan("noise_mix_median", "canonical", R(0))


# ---- test_v0 (lib/model/test.py as-is) -----------------------------------------------------
def test_test_v0_gaussian_picks_random_level_and_returns_float64():
    levels = set()
    for s in range(60):
        p = ns.plan("gaussian_median_var0.1", "test_v0", R(s))  # test.py:1678-1690
        assert p.out_dtype == "f64" and len(p.steps) == 1  # median hook is dead in test.py
        levels.add(p.steps[0].args[0])
    assert levels == {0.1, 1.0, 1.5}


def test_test_v0_sap_and_quant_are_original():
    for spec in ("sap_var0.4", "sap_median_var0.2", "quant_var3"):
        assert ops(ns.plan(spec, "test_v0", R(0))) == [("noise", "original")]  # test.py:1691-1697


def test_test_v0_poisson_ignores_denoiser_except_wavelet():
    assert ops(ns.plan("poisson_median", "test_v0", R(0))) == [("noise", "poisson"), ("cast_u8", "u8")]
    p = ns.plan("poisson_wavelet", "test_v0", R(0))
    # closure runs poisson (no denoise: noise_type forced to 'poisson'), then the live hook
    assert ops(p)[-1] == ("filter", "wavelet", "bior1.5", None)


def test_test_v0_unknown_falls_to_gaussian_mean_on_float():
    p = ns.plan("anything", "test_v0", R(0))  # test.py:1757-1768
    assert ops(p) == [("noise", "gaussian", 0.1), ("filter", "mean", 3)] and p.out_dtype == "f64"


def test_test_v0_curvelet_discarded():
    assert ops(ns.plan("curvelet", "test_v0", R(0))) == [("noise", "original")]


def test_test_v0_mix_pool_and_bloom():
    seen = set()
    for s in range(400):
        p = ns.plan("noise_mix_var_low", "test_v0", R(s))  # quant included: no draw raises
        seen.add(p.noise_type)
    assert {"bloom", "sap_var0.2", "quant_var3"} <= seen
    assert ops(ns.plan("bloom", "test_v0", R(0))) == [("noise", "bloom")]


# ---- train_v0 (lib/roi_data_layer/minibatch.py as-is) --------------------------------------
def test_train_v0_double_filtering():
    p = ns.plan("speckle_mean_var1.0", "train_v0", R(0))  # closure mean + hook mean
    assert ops(p) == [("noise", "speckle", 1.0), ("cast_u8", "u8"), ("filter", "mean", 3),
                      ("filter", "mean", 3)]


def test_train_v0_plain_branches_float64_and_sap_quirk():
    p = ns.plan("sap_var0.8", "train_v0", R(0))
    assert ops(p) == [("noise", "sap", 0.6)] and p.out_dtype == "f64"  # minibatch.py:367
    p = ns.plan("sap_median_var0.8", "train_v0", R(0))
    assert ops(p)[0] == ("noise", "sap", 0.8)
    assert ns.plan("poisson", "train_v0", R(0)).out_dtype == "f64"


def test_train_v0_hook_on_float64_mean_and_failures():
    for s in range(20):
        p = ns.plan("gaussian_mean_var0.1", "train_v0", R(s))
        assert p.out_dtype == "f64" and ops(p)[-1] == ("filter", "mean", 3)
    with pytest.raises(RuntimeError):
        ns.plan("speckle_median_var0.5", "train_v0", R(0)) if False else \
            ns.plan("gaussian_median_var0.5", "train_v0", R(0))
    with pytest.raises(NameError):
        ns.plan("bloom", "train_v0", R(0))  # add_bloom uses `math` without importing it
    with pytest.raises(AttributeError):
        ns.plan("speckle_var9.9", "train_v0", R(0))  # closure returns [] -> .astype fails


def test_train_v0_mix_bloom_runs_shader():
    for s in range(400):
        p = ns.plan("noise_mix_var_low", "train_v0", R(s))
        if p.noise_type == "bloom":
            assert ops(p) == [("noise", "shader")]  # minibatch.py:1571-1572
            return
    pytest.fail("bloom never drawn")


def test_unknown_level_unbound_in_test_v0():
    with pytest.raises(UnboundLocalError):
        ns.plan("speckle_var9.9", "test_v0", R(0))


def test_quant_and_additive_noises_planned():
    # MiniBatchKMeans(n_clusters=k) in LAB, then LAB->BGR: u8 (minibatch.py:492-667)
    assert ops(ns.plan("quant_var3", "train_v0", R(0))) == [("noise", "quant", 3)]
    assert ops(ns.plan("quant_var10", "canonical", R(0))) == [("noise", "quant", 10)]
    assert ops(ns.plan("quant_median_var7", "canonical", R(0))) == [
        ("noise", "quant", 7), ("filter", "median", 3)]
    assert ops(ns.plan("quant_wavelet_var10", "canonical", R(0))) == [
        ("noise", "quant", 10), ("filter", "wavelet", "bior1.5", None)]
    # train_v0: closure median + post-hook median (double filtering, as for the other noises)
    assert ops(ns.plan("quant_median_var3", "train_v0", R(0))) == [
        ("noise", "quant", 3), ("filter", "median", 3), ("filter", "median", 3)]
    with pytest.raises(AttributeError):
        ns.plan("quant_var5", "train_v0", R(0))  # `im = []` returned (minibatch.py:493)
    for s in range(50):  # every mix list resolves (quant was the last unplanned type)
        for key in ("var_low", "var_medium", "var_high", "var_all"):
            for mode in ("test_v0", "train_v0", "canonical"):
                ns.plan(f"noise_mix_{key}", mode, R(s))
    assert ops(ns.plan("uniform_var0.6", "train_v0", R(0))) == [("noise", "uniform", 0.6)]
    assert ns.plan("uniform_var0.6", "train_v0", R(0)).out_dtype == "f64"  # minibatch.py:787
    assert ops(ns.plan("gamma_var0.2", "test_v0", R(0))) == [("noise", "gamma", 0.2), ("cast_u8", "u8")]
    assert ops(ns.plan("rayleigh_median_var0.3", "canonical", R(0))) == [
        ("noise", "rayleigh", 0.3), ("cast_u8", "u8"), ("filter", "median", 3)]
    # brownian: cv2.add(img, U8(255 B)) is u8; 'var0.09' is not read as 'var0.9'
    assert ops(ns.plan("brownian_var0.09", "canonical", R(0))) == [("noise", "brownian", 0.09)]
    assert ops(ns.plan("brownian_wavelet_var0.009", "canonical", R(0))) == [
        ("noise", "brownian", 0.009), ("filter", "wavelet", "bior1.5", None)]
    # additive wavelet branches denoise the unclipped float sum (no U8 before the wavelet)
    assert ops(ns.plan("uniform_wavelet_var1.2", "canonical", R(0))) == [
        ("noise", "uniform", 1.2), ("filter", "wavelet", "bior1.5", None)]


def test_periodic_amplitude():
    import math
    assert ns.periodic_amplitude("pi", 10) == math.pi
    assert ns.periodic_amplitude("size", 1800000) == 1800000.0
    assert ns.periodic_amplitude(100.0, 5) == 100.0
