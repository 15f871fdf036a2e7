"""CPU oracle for theoretical isotope patterns.

TEST INFRASTRUCTURE ONLY.  Nothing in ``sm_distributed_amd`` imports this module; ``tests/`` use it as
the checker of the native calculator (``smg_isotope_centroids`` in ``libsmg.so``).

Reference call site: ``sm/engine/isocalc_wrapper.py:37-70`` -- ``complete_isodist(parseSumFormula(sf +
adduct), sigma, charge, pts_per_mz, centroid_kwargs={'weighted_bins': 5})``, then the first six centroids
in m/z order.  The arithmetic lives in third-party packages that are NOT in /root/reference and not in
this image (``cpyMSpec`` ``legacy_interface.complete_isodist``, ``pyMSpec`` ``parseSumFormula`` /
``centroid_detection.gradient``; ``requirements.txt:1-2``).  Every reference test that touches them patches
them out (``sm/engine/tests/test_isocalc_wrapper.py:9``, ``test_theor_peaks_gen.py:17``), so **parity is
unpinned** for the numbers: this module is the contract, restated from the published algorithm (isotopic
fine structure -> Gaussian profile -> gradient centroids):

1. ``parse_sum_formula``: elements ``[A-Z][a-z]*`` with optional counts, nested ``( )`` groups with a
   multiplier, ``+`` / ``-`` between sub-formulas (``"C6H12O6" + "-H"``); an unknown element, a malformed
   string or a negative final count is an invalid formula (pyMSpec ``InvalidFormulaError``; the wrapper
   then returns empty centroids, ``isocalc_wrapper.py:64-65``).
2. Fine structure: per element (in symbol order) the n-fold isotope distribution by binary powering, then
   the product over elements; every product drops peaks below ``PRUNE`` x its maximum and merges runs of
   peaks whose consecutive masses differ by <= ``MERGE_TOL`` Da (abundance-weighted mean mass).  Peaks
   below ``cutoff_perc`` % of the maximum are then dropped (pyMSpec ``perfect_pattern`` default 0.1 %).
3. Charge: ``mz = (m - z * m_e) / |z|`` for z != 0 (a positive ion lost z electrons); z = 0 keeps masses.
4. Profile: a Gaussian of FWHM ``sigma / 2.35482`` (standard deviation s = FWHM / 2.35482) on the grid
   ``x_j = j / pts_per_mz``, each peak evaluated over ``|x - m| <= 6 s``, peaks added in ascending mass.
   Evidence for reading ``isocalc_sigma`` as 2.35482 x FWHM: the reference's resolving-power table
   ``scripts/generate_ds_config.py:54-85`` sets ``sigma = 2.35482 * fwhm`` and ``pts_per_mz = 5 / fwhm``
   (five grid points per FWHM) for every entry.
5. Centroids (pyMSpec ``gradient``): every grid point with ``y[j-1] < y[j] >= y[j+1]`` and ``y[j] > 0``;
   m/z = intensity-weighted mean of ``x`` over ``j-w .. j+w`` (w = ``weighted_bins``), intensity = ``y[j]``;
   intensities scaled to a maximum of 100; ascending m/z.

Physical constants: IUPAC/NIST isotope masses and representative abundances (``ISOTOPES``); the native
calculator carries the same table.
"""
from __future__ import annotations

import re

import numpy as np

ELECTRON_MASS = 0.00054857990946
FWHM_PER_SIGMA = 2.3548200450309493
PRUNE = 1e-9
MERGE_TOL = 1e-6
TRUNC_S = 6.0
CUTOFF_PERC = 0.1

# element -> ((mass, abundance), ...), ascending mass
ISOTOPES = {
    "H": ((1.00782503207, 0.999885), (2.0141017778, 0.000115)),
    "He": ((3.0160293191, 1.34e-06), (4.00260325415, 0.99999866)),
    "Li": ((6.015122795, 0.0759), (7.01600455, 0.9241)),
    "B": ((10.0129370, 0.199), (11.0093054, 0.801)),
    "C": ((12.0, 0.9893), (13.0033548378, 0.0107)),
    "N": ((14.0030740048, 0.99636), (15.0001088982, 0.00364)),
    "O": ((15.99491461956, 0.99757), (16.99913170, 0.00038), (17.9991610, 0.00205)),
    "F": ((18.99840322, 1.0),),
    "Na": ((22.9897692809, 1.0),),
    "Mg": ((23.985041700, 0.7899), (24.98583692, 0.1000), (25.982592929, 0.1101)),
    "Al": ((26.98153863, 1.0),),
    "Si": ((27.9769265325, 0.92223), (28.976494700, 0.04685), (29.97377017, 0.03092)),
    "P": ((30.97376163, 1.0),),
    "S": ((31.97207100, 0.9499), (32.97145876, 0.0075), (33.96786690, 0.0425), (35.96708076, 0.0001)),
    "Cl": ((34.96885268, 0.7576), (36.96590259, 0.2424)),
    "K": ((38.96370668, 0.932581), (39.96399848, 0.000117), (40.96182576, 0.067302)),
    "Ca": ((39.96259098, 0.96941), (41.95861801, 0.00647), (42.9587666, 0.00135), (43.9554818, 0.02086),
           (45.9536926, 4e-05), (47.952534, 0.00187)),
    "Mn": ((54.9380451, 1.0),),
    "Fe": ((53.9396105, 0.05845), (55.9349375, 0.91754), (56.9353940, 0.02119), (57.9332756, 0.00282)),
    "Co": ((58.9331950, 1.0),),
    "Ni": ((57.9353429, 0.680769), (59.9307864, 0.262231), (60.9310560, 0.011399), (61.9283451, 0.036345),
           (63.9279660, 0.009256)),
    "Cu": ((62.9295975, 0.6915), (64.9277895, 0.3085)),
    "Zn": ((63.9291422, 0.48268), (65.9260334, 0.27975), (66.9271273, 0.04102), (67.9248442, 0.19024),
           (69.9253193, 0.00631)),
    "As": ((74.9215965, 1.0),),
    "Se": ((73.9224764, 0.0089), (75.9192136, 0.0937), (76.9199140, 0.0763), (77.9173091, 0.2377),
           (79.9165213, 0.4961), (81.9166994, 0.0873)),
    "Br": ((78.9183371, 0.5069), (80.9162906, 0.4931)),
    "I": ((126.904473, 1.0),),
    "Au": ((196.9665687, 1.0),),
}


class InvalidFormulaError(ValueError):
    pass


_TOKEN = re.compile(r"([A-Z][a-z]*|\(|\)|\d+|[+-])")


def parse_sum_formula(s) -> dict:
    """Element counts of ``s`` (module doc, item 1); raises InvalidFormulaError."""
    if not isinstance(s, str) or not s:
        raise InvalidFormulaError(f"invalid sum formula {s!r}")
    toks = _TOKEN.findall(s)
    if "".join(toks) != s:
        raise InvalidFormulaError(f"unexpected characters in {s!r}")
    pos = 0

    def group():  # (element | '(' group ')') [count] ... up to ')' / sign / end
        nonlocal pos
        out: dict = {}
        n_items = 0
        while pos < len(toks) and toks[pos] not in (")", "+", "-"):
            t = toks[pos]
            if t == "(":
                pos += 1
                sub = group()
                if pos >= len(toks) or toks[pos] != ")":
                    raise InvalidFormulaError(f"unbalanced parenthesis in {s!r}")
                pos += 1
            elif t[0].isupper():
                if t not in ISOTOPES:
                    raise InvalidFormulaError(f"unknown element {t!r} in {s!r}")
                sub = {t: 1}
                pos += 1
            else:
                raise InvalidFormulaError(f"misplaced count in {s!r}")
            mult = 1
            if pos < len(toks) and toks[pos].isdigit():
                mult = int(toks[pos])
                pos += 1
            for e, c in sub.items():
                out[e] = out.get(e, 0) + c * mult
            n_items += 1
        if n_items == 0:
            raise InvalidFormulaError(f"empty group in {s!r}")
        return out

    total: dict = {}
    sign = 1
    if toks[0] in ("+", "-"):
        sign = -1 if toks[0] == "-" else 1
        pos = 1
    while True:
        for e, c in group().items():
            total[e] = total.get(e, 0) + sign * c
        if pos >= len(toks):
            break
        if toks[pos] not in ("+", "-"):
            raise InvalidFormulaError(f"unbalanced parenthesis in {s!r}")
        sign = -1 if toks[pos] == "-" else 1
        pos += 1
        if pos >= len(toks):
            raise InvalidFormulaError(f"dangling sign in {s!r}")
    if any(c < 0 for c in total.values()):
        raise InvalidFormulaError(f"negative element count in {s!r}")
    total = {e: c for e, c in total.items() if c > 0}
    if not total:
        raise InvalidFormulaError(f"no atoms in {s!r}")
    return total


def _convolve(am, ap, bm, bp):
    m = (am[:, None] + bm[None, :]).ravel()
    p = (ap[:, None] * bp[None, :]).ravel()
    keep = p >= PRUNE * p.max()
    m, p = m[keep], p[keep]
    o = np.argsort(m, kind="stable")
    m, p = m[o], p[o]
    # merge runs whose consecutive masses differ by <= MERGE_TOL (abundance-weighted mean mass)
    starts = np.concatenate(([0], np.nonzero(np.diff(m) > MERGE_TOL)[0] + 1))
    ps = np.add.reduceat(p, starts)
    ms = np.add.reduceat(m * p, starts) / ps
    return ms, ps


def _element_power(el, n):
    iso = ISOTOPES[el]
    bm = np.array([x[0] for x in iso])
    bp = np.array([x[1] for x in iso])
    rm, rp = np.array([0.0]), np.array([1.0])
    while n:
        if n & 1:
            rm, rp = _convolve(rm, rp, bm, bp)
        n >>= 1
        if n:
            bm, bp = _convolve(bm, bp, bm, bp)
    return rm, rp


def fine_structure(counts: dict):
    """(masses, abundances) of the molecule, ascending mass (module doc, item 2, before the cutoff)."""
    m, p = np.array([0.0]), np.array([1.0])
    for el in sorted(counts):
        em, ep = _element_power(el, counts[el])
        m, p = _convolve(m, p, em, ep)
    return m, p


def isotope_centroids(sf_adduct: str, charge: int, sigma: float, pts_per_mz: int, weighted_bins: int = 5,
                      cutoff_perc: float = CUTOFF_PERC):
    """All centroids (mzs, ints) of ``sf_adduct`` in m/z order, max intensity 100 (module doc, 1-5)."""
    counts = parse_sum_formula(sf_adduct)
    m, p = fine_structure(counts)
    keep = p >= cutoff_perc / 100.0 * p.max()
    m, p = m[keep], p[keep]
    if charge:
        m = (m - charge * ELECTRON_MASS) / abs(charge)
    s = sigma / FWHM_PER_SIGMA / FWHM_PER_SIGMA
    lo = np.ceil((m - TRUNC_S * s) * pts_per_mz).astype(np.int64)
    hi = np.floor((m + TRUNC_S * s) * pts_per_mz).astype(np.int64)
    j0 = int(lo.min()) - weighted_bins - 1
    j1 = int(hi.max()) + weighted_bins + 1
    x = np.arange(j0, j1 + 1, dtype=np.int64) / float(pts_per_mz)
    y = np.zeros(len(x))
    for i in range(len(m)):  # ascending mass
        a, b = lo[i] - j0, hi[i] - j0 + 1
        d = x[a:b] - m[i]
        y[a:b] += p[i] * np.exp(-(d * d) / (2.0 * s * s))
    mzs, ints = [], []
    for j in range(1, len(y) - 1):
        if y[j] > 0.0 and y[j - 1] < y[j] and y[j] >= y[j + 1]:
            a, b = j - weighted_bins, j + weighted_bins + 1
            mzs.append(float(np.sum(x[a:b] * y[a:b]) / np.sum(y[a:b])))
            ints.append(float(y[j]))
    mzs, ints = np.array(mzs), np.array(ints)
    ints = ints * (100.0 / ints.max())
    return mzs, ints


def monoisotopic_mz(sf_adduct: str, charge: int) -> float:
    """m/z of the all-lightest-isotope species (the monoisotopic peak of organic ions)."""
    counts = parse_sum_formula(sf_adduct)
    m = sum(c * ISOTOPES[e][0][0] for e, c in counts.items())
    return (m - charge * ELECTRON_MASS) / abs(charge) if charge else m
