"""The `--noise` plugin surface: noise-spec string -> per-image plan of kernel steps.

The reference dispatches on Python substring tests of one string (README.md:82-107), with two
diverging copies of the logic:

  test_v0   lib/model/test.py:193-1607 (closures), 1611-1677 (mix), 1678-1785 (single),
            1787-1831 (post hook: only 'wavelet' is live)
  train_v0  lib/roi_data_layer/minibatch.py:87-1516 (closures), 1518-1574 (mix),
            1575-1634 (single), 1636-1673 (post hook: every denoiser live -> double filtering)
  canonical the README grammar with the in-branch semantics (one noise, at most one denoise)

`plan(noise, mode, rng)` resolves one image's recipe exactly as the chosen copy does, including
its as-is quirks (test_v0 'sap'/'quant' add no noise, gaussian ignores the level and returns
float64, unknown strings fall to gaussian_var0.1 + 3x3 mean; train_v0 maps sap var0.8 to amount
0.6, plain noises return float64, 'bloom' in a mix runs the shader, median on float64 raises).
The reference's failure modes are reproduced as the same Python exception types.

A plan is a tuple of Steps executed by idn.pipeline on device tensors.
"""
from __future__ import annotations

import math
import random as _random
from dataclasses import dataclass, field
from typing import Optional, Tuple

MODES = ("canonical", "test_v0", "train_v0")
DENOISERS = ("wavelet", "gaus_blur", "mean", "median", "bilateral")  # reference test order
NOISES = ("gaussian", "sap", "speckle", "poisson", "quant", "uniform", "periodic", "brownian",
          "gamma", "rayleigh")

# level tokens in the order the reference tests them (first substring match wins)
LEVELS = {
    "gaussian": (("var0.1", 0.1), ("var1.0", 1.0), ("var1.5", 1.5)),
    "sap": (("var0.2", 0.2), ("var0.4", 0.4), ("var0.8", 0.8)),
    "speckle": (("var0.5", 0.5), ("var1.0", 1.0), ("var2.0", 2.0)),
    "periodic": (("var3.14", "pi"), ("var100", 100.0), ("varsize", "size")),
    # the reference's own additive noises (test.py:767-1572, minibatch.py:669-1490)
    "uniform": (("var0.2", 0.2), ("var0.6", 0.6), ("var1.2", 1.2)),        # high
    "brownian": (("var0.9", 0.9), ("var0.09", 0.09), ("var0.009", 0.009)),  # dt
    "gamma": (("var0.05", 0.05), ("var0.1", 0.1), ("var0.2", 0.2)),         # scale
    "rayleigh": (("var0.1", 0.1), ("var0.2", 0.2), ("var0.3", 0.3)),        # scale
    # MiniBatchKMeans(n_clusters=k) colour quantisation in LAB (test.py:592-765,
    # minibatch.py:492-667); tested in this order, so 'var10' is reached only without var3/var7
    "quant": (("var3", 3), ("var7", 7), ("var10", 10)),                       # clusters
}
ADDITIVE = ("uniform", "gamma", "rayleigh")  # float64 x + noise, unclipped (cv2.add on floats)

# reference in-branch denoiser parameters (test.py:220,241,259,272-274 / minibatch.py likewise)
BILATERAL_REF = (9, 20.0, 100.0)  # diameter, sigmaColor, sigmaSpace, BORDER_CONSTANT
KSIZE_REF = 3

MIX_TEST = {  # lib/model/test.py:1613-1639
    "var_low": ["gaussian_var0.1", "poisson", "speckle_var0.5", "sap_var0.2", "uniform_var0.2",
                "gamma_var0.05", "rayleigh_var0.1", "periodic_var3.14", "brownian_var0.9",
                "quant_var3", "original", "bloom", "shader"],
    "var_medium": ["gaussian_var1.0", "poisson", "speckle_var1.0", "sap_var0.4", "uniform_var0.6",
                   "gamma_var0.1", "rayleigh_var0.2", "periodic_var100", "brownian_var0.09",
                   "quant_var7", "original", "shader", "bloom"],
    "var_high": ["gaussian_var1.5", "poisson", "speckle_var2.0", "sap_var0.8", "uniform_var1.2",
                 "gamma_var0.2", "rayleigh_var0.3", "periodic_varsize", "brownian_var0.009",
                 "quant_var10", "original", "shader", "bloom"],
    "var_all": ["gaussian_var0.1", "poisson", "speckle_var0.5", "sap_var0.2", "uniform_var0.2",
                "gamma_var0.05", "gamma_var0.05", "rayleigh_var0.2", "rayleigh_var0.1",
                "periodic_var3.14", "brownian_var0.9", "quant_var3", "gamma_var0.1",
                "rayleigh_var0.1", "gaussian_var1.0", "poisson", "speckle_var1.0", "sap_var0.4",
                "uniform_var0.6", "gamma_var0.1", "shader", "original", "shader", "bloom",
                "rayleigh_var0.2", "periodic_var100", "brownian_var0.09", "quant_var7",
                "gaussian_var1.5", "poisson", "speckle_var2.0", "sap_var0.8", "uniform_var1.2",
                "gamma_var0.2", "shader", "original", "rayleigh_var0.3", "periodic_varsize",
                "brownian_var0.009", "quant_var10", "original", "shader"],
}
MIX_TRAIN = {  # lib/roi_data_layer/minibatch.py:1519-1547
    "var_low": ["gaussian_var0.1", "poisson", "speckle_var0.5", "sap_var0.2", "uniform_var0.2",
                "gamma_var0.05", "rayleigh_var0.1", "periodic_var3.14", "brownian_var0.9",
                "quant_var10", "original", "bloom", "shader"],
    "var_medium": ["gaussian_var1.0", "poisson", "speckle_var1.0", "sap_var0.4", "uniform_var0.6",
                   "gamma_var0.1", "rayleigh_var0.2", "periodic_var100", "brownian_var0.09",
                   "quant_var7", "original", "bloom", "shader"],
    "var_high": ["gaussian_var1.5", "poisson", "speckle_var2.0", "sap_var0.8", "uniform_var1.2",
                 "gamma_var0.2", "rayleigh_var0.3", "periodic_varsize", "brownian_var0.009",
                 "quant_var3", "original", "bloom", "shader"],
    "var_all": ["gaussian_var0.1", "poisson", "speckle_var0.5", "sap_var0.2", "uniform_var0.2",
                "gamma_var0.05", "rayleigh_var0.1", "periodic_var3.14", "brownian_var0.9",
                "quant_var3", "shader", "bloom", "gaussian_var1.0", "poisson", "speckle_var1.0",
                "sap_var0.4", "uniform_var0.6", "gamma_var0.1", "original", "shader", "bloom",
                "rayleigh_var0.2", "periodic_var100", "brownian_var0.09", "quant_var7",
                "gaussian_var1.5", "poisson", "speckle_var2.0", "sap_var0.8", "uniform_var1.2",
                "gamma_var0.2", "rayleigh_var0.3", "periodic_varsize", "brownian_var0.009",
                "quant_var10", "original", "shader", "bloom"],
}
MIX_KEYS = ("var_low", "var_medium", "var_high", "var_all")  # reference test order


@dataclass(frozen=True)
class Step:
    """One kernel step.  op in:
    noise:    ('gaussian', var) ('speckle', var) ('sap', amount) ('poisson',) ('periodic', amp)
              ('quant', k) ('original',) ('bloom', [circles]) ('shader',)
    cast_u8:  U8(255*x) of a float64 image
    filter:   ('gaus_blur', k) ('mean', k) ('median', k) ('bilateral', d, sc, ss)
              ('wavelet', wavelet, levels)
    """
    kind: str                 # 'noise' | 'cast_u8' | 'filter'
    op: str
    args: Tuple = ()


@dataclass(frozen=True)
class Plan:
    spec: str                 # the user's noise string
    noise_type: str           # the resolved (possibly randomly chosen) noise type
    steps: Tuple[Step, ...]
    out_dtype: str            # 'u8' or 'f64' (what the reference hands to the blob builder)
    log: Tuple[str, ...] = field(default=())  # the reference's print()s, for tracing


class ReferenceError_(Exception):
    """Base for reproduced reference failures (never raised directly)."""


def _level(noise: str, noise_type: str):
    for tok, val in LEVELS[noise]:
        if tok in noise_type:
            return tok, val
    return None, None


def _denoiser(noise: str, noise_type: str) -> Optional[str]:
    for den in DENOISERS:
        if f"{noise}_{den}" in noise_type:
            return den
    return None


def _filter_step(den: str) -> Step:
    if den == "wavelet":
        return Step("filter", "wavelet", ("bior1.5", None))
    if den == "gaus_blur":
        return Step("filter", "gaus_blur", (KSIZE_REF,))
    if den == "mean":
        return Step("filter", "mean", (KSIZE_REF,))
    if den == "median":
        return Step("filter", "median", (KSIZE_REF,))
    return Step("filter", "bilateral", BILATERAL_REF)


def _unbound():
    # the closure's local `im` is returned without being assigned
    raise UnboundLocalError("local variable 'im' referenced before assignment "
                            "(noise level token not recognised, as in the reference)")


def _noise_branch(noise: str, noise_type: str, mode: str):
    """add_<noise>_noise(noise_type): returns (steps, out_dtype) of one closure."""
    den = _denoiser(noise, noise_type)
    if noise == "poisson":
        noise_step = Step("noise", "poisson")
        tok = "poisson"
    else:
        tok, val = _level(noise, noise_type)
        if tok is None:
            if mode == "train_v0":
                return None, "empty"  # `im = []` is returned; prep_im_for_blob fails later
            _unbound()
        if noise == "sap" and mode == "train_v0" and tok == "var0.8" and den is None:
            val = 0.6  # minibatch.py:367: the plain var0.8 branch draws amount=0.6
        noise_step = Step("noise", "sap" if noise == "sap" else noise, (val,))
    steps = [noise_step]
    if noise == "quant":
        # cvtColor(LAB2BGR) of the quantised image is already u8; every denoiser (wavelet
        # included) runs on it (test.py:600-757)
        if den is not None:
            steps.append(_filter_step(den))
        return steps, "u8"
    if noise == "brownian":
        # cv2.add(img, U8(255 * B)) is already u8 (test.py:1095-1124); denoisers run on it
        if den is not None:
            steps.append(_filter_step(den))
        return steps, "u8"
    if noise in ADDITIVE:
        if den == "wavelet":  # denoise_wavelet on the unclipped float64 sum
            return steps + [_filter_step("wavelet")], "u8"
        if den is not None:
            return steps + [Step("cast_u8", "u8"), _filter_step(den)], "u8"
        if mode == "train_v0":  # minibatch.py:787,1324,1464: `im = uniform_noise` (float64)
            return steps, "f64"
        return steps + [Step("cast_u8", "u8")], "u8"
    if noise == "periodic":
        # cv2.add(img, pattern) is already u8; denoisers then run on it
        if den is not None:
            steps.append(_filter_step(den))
        return steps, "u8"
    if den == "wavelet":
        # gaussian / sap / speckle feed the float64 noisy image to denoise_wavelet; poisson first
        # casts it to u8 (test.py:315-316)
        if noise == "poisson":
            steps.append(Step("cast_u8", "u8"))
        steps.append(_filter_step("wavelet"))
        return steps, "u8"
    if den is not None:
        steps.append(Step("cast_u8", "u8"))
        steps.append(_filter_step(den))
        return steps, "u8"
    # plain branch
    plain_f64 = {
        "test_v0": ("gaussian",),
        "train_v0": ("gaussian", "poisson", "sap", "speckle"),
        "canonical": (),
    }[mode]
    if noise in plain_f64:
        return steps, "f64"
    steps.append(Step("cast_u8", "u8"))
    return steps, "u8"


def _closure(noise_type: str, mode: str, top_level: bool):
    """dispatch one (resolved) noise type to its closure."""
    for noise in ("gaussian", "poisson", "sap", "speckle", "periodic", "brownian", "quant",
                  "uniform", "gamma", "rayleigh"):
        if noise in noise_type:
            if noise == "quant" and mode == "test_v0" and top_level:
                return [Step("noise", "original")], "u8"  # test.py:1719-1725 adds no noise
            if mode == "test_v0" and top_level and noise == "sap":
                return [Step("noise", "original")], "u8"  # test.py:1691-1697
            return _noise_branch(noise, noise_type, mode)
    if "bloom" in noise_type:
        if mode == "train_v0" and not top_level:
            return [Step("noise", "shader")], "u8"  # minibatch.py:1571-1572
        if mode == "train_v0":
            raise NameError("name 'math' is not defined (minibatch.py add_bloom, as in the reference)")
        return [Step("noise", "bloom")], "u8"
    if "shader" in noise_type:
        return [Step("noise", "shader")], "u8"
    return [Step("noise", "original")], "u8"


def _post_hook(noise: str, steps, out_dtype: str, mode: str):
    """the post-dispatch denoise hook (test.py:1787-1831, minibatch.py:1636-1673)."""
    if mode == "canonical":
        return steps, out_dtype
    for den in ("gaus_blur", "mean", "median", "wavelet", "bilateral", "curvelet"):
        if den in noise:
            break
    else:
        return steps, out_dtype
    if den == "curvelet":
        if mode == "test_v0":
            return [Step("noise", "original")], "u8"  # test.py:1831 discards the subprocess result
        raise NotImplementedError("curvelet denoising (subprocess + curvelops FDCT3D) is out of scope")
    if mode == "test_v0" and den != "wavelet":
        return steps, out_dtype  # test.py: only the wavelet hook is live
    if den == "wavelet":
        return steps + [_filter_step("wavelet")], "u8"
    if den == "median" and out_dtype == "f64":
        raise RuntimeError("cv2.error: medianBlur does not support float64 input "
                           "(minibatch.py:1647, as in the reference)")
    if den == "bilateral" and out_dtype == "f64":
        raise RuntimeError("cv2.error: bilateralFilter supports only 8u and 32f images "
                           "(minibatch.py:1662, as in the reference)")
    return steps + [_filter_step(den)], out_dtype


def plan(noise: str, mode: str = "canonical", rng: Optional[_random.Random] = None,
         hw: Optional[Tuple[int, int]] = None) -> Plan:
    """Resolve the recipe for ONE image.  `rng` provides random.choice (the reference uses the
    unseeded global `random`); pass a seeded random.Random for reproducible batches.

    hw = (H, W) of the image: a `bloom` step then carries its add_sun_flare circles, drawn from
    `rng` right after the noise-type choice -- the order the reference's loop draws them in
    (test.py:1590-1617: random.choice, then Automold's random.uniform / randint calls) -- so the
    draws belong to the plan, not to whichever process later executes it."""
    if mode not in MODES:
        raise ValueError(f"mode must be one of {MODES}")
    rng = rng or _random
    p = _plan_canonical(noise, rng) if mode == "canonical" else _plan_mode(noise, mode, rng)
    if hw is not None and any(st.op == "bloom" and not st.args for st in p.steps):
        p = _with_bloom_draws(p, hw, rng)
    return p


def _with_bloom_draws(p: Plan, hw: Tuple[int, int], rng) -> Plan:
    from . import automold
    circ, wts = automold.sun_flare_circles(int(hw[0]), int(hw[1]), flare_center=(100, 100),
                                           angle=-math.pi / 4, rng=rng)
    args = (tuple(tuple(int(v) for v in r) for r in circ),
            tuple(tuple(float(v) for v in r) for r in wts))
    steps = tuple(Step("noise", "bloom", args) if (st.op == "bloom" and not st.args) else st
                  for st in p.steps)
    return Plan(p.spec, p.noise_type, steps, p.out_dtype, p.log)


def _plan_mode(noise: str, mode: str, rng) -> Plan:
    mix = MIX_TEST if mode == "test_v0" else MIX_TRAIN
    if "mix" in noise:
        for key in MIX_KEYS:
            if key in noise:
                noise_type = rng.choice(mix[key])
                break
        else:
            raise UnboundLocalError("local variable 'noise_type' referenced before assignment "
                                    "(mix spec without var_low/medium/high/all, as in the reference)")
        steps, out = _closure(noise_type, mode, top_level=False)
    elif "gaussian" in noise:
        noise_type = rng.choice(["gaussian_var0.1", "gaussian_var1.0", "gaussian_var1.5"])
        steps, out = _closure(noise_type, mode, top_level=True)
    elif "curvelet" in noise and not any(n in noise for n in NOISES):
        noise_type = noise
        steps, out = [Step("noise", "original")], "u8"
        if mode == "train_v0":
            raise NotImplementedError("curvelet denoising (subprocess + curvelops) is out of scope")
    elif any(n in noise for n in ("poisson", "sap", "speckle", "periodic", "brownian", "quant",
                                  "uniform", "gamma", "rayleigh", "bloom", "shader")):
        noise_type = "poisson" if (mode == "test_v0" and "poisson" in noise) else noise
        steps, out = _closure(noise_type, mode, top_level=True)
    else:
        if mode == "test_v0":
            # test.py:1757-1768: gaussian_var0.1 (float64) then cv2.blur 3x3 on the float image
            noise_type = "gaussian_var0.1"
            steps, out = [Step("noise", "gaussian", (0.1,)), Step("filter", "mean", (3,))], "f64"
        else:
            noise_type = "original"
            steps, out = [Step("noise", "original")], "u8"
    if out == "empty":
        raise AttributeError("'list' object has no attribute 'astype' (the closure returned [] "
                             "for an unrecognised level, as in the reference)")
    steps, out = _post_hook(noise, list(steps), out, mode)
    return Plan(noise, noise_type, tuple(steps), out)


def _plan_canonical(noise: str, rng) -> Plan:
    """README grammar: {noise}[_{denoise}]_var{level} | poisson[_{denoise}] |
    noise_mix_var_{low|medium|high|all}[_{denoise}] | original | bloom | shader."""
    s = noise.strip()
    den = None
    for d in DENOISERS:
        if f"_{d}" in s:
            den = d
    if s.startswith("noise_mix"):
        key = next((k for k in ("var_all", "var_low", "var_medium", "var_high") if k in s), None)
        if key is None:
            raise ValueError(f"mix spec {noise!r} needs var_low / var_medium / var_high / var_all")
        pool = [t for t in MIX_TEST[key] if t.split("_")[0] in
                ("gaussian", "poisson", "speckle", "sap", "periodic", "original", "quant") +
                ADDITIVE + ("brownian",)]
        base = rng.choice(pool)
        noise_type = base if den is None else _insert_denoiser(base, den)
        return _plan_canonical(noise_type, rng)._replace_spec(noise)
    if s in ("original", "bloom", "shader"):
        return Plan(noise, s, (Step("noise", s),), "u8")
    if s.startswith("original_") and den is not None:
        return Plan(noise, s, (Step("noise", "original"), _filter_step(den)), "u8")
    head = s.split("_")[0]
    if head not in ("gaussian", "sap", "speckle", "poisson", "periodic", "quant") + ADDITIVE + \
            ("brownian",):
        raise ValueError(f"unknown or unsupported noise spec {noise!r}")
    steps, out = _noise_branch(head, s, "canonical")
    return Plan(noise, s, tuple(steps), out)


def _insert_denoiser(noise_type: str, den: str) -> str:
    head, _, rest = noise_type.partition("_")
    return f"{head}_{den}" + (f"_{rest}" if rest else "")


def _replace_spec(self: Plan, spec: str) -> Plan:
    return Plan(spec, self.noise_type, self.steps, self.out_dtype, self.log)


Plan._replace_spec = _replace_spec  # type: ignore[attr-defined]


def periodic_amplitude(val, size: int) -> float:
    if val == "pi":
        return math.pi
    if val == "size":
        return float(size)
    return float(val)
