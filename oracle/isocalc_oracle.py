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
    # the remaining decoy-adduct elements of fdr.py:8 (NIST isotope masses, IUPAC representative abundances)
    "Be": ((9.0121822, 1.0),),
    "Ne": ((19.9924401754, 0.9048), (20.99384668, 0.0027), (21.991385114, 0.0925)),
    "Ar": ((35.967545106, 0.003365), (37.9627324, 0.000632), (39.9623831225, 0.996003)),
    "Sc": ((44.9559119, 1.0),),
    "Ti": ((45.9526316, 0.0825), (46.9517631, 0.0744), (47.9479463, 0.7372), (48.94787, 0.0541), (49.9447912, 0.0518)),
    "V": ((49.9471585, 0.0025), (50.9439595, 0.9975)),
    "Cr": ((49.9460442, 0.04345), (51.9405075, 0.83789), (52.9406494, 0.09501), (53.9388804, 0.02365)),
    "Ga": ((68.9255736, 0.60108), (70.9247013, 0.39892)),
    "Ge": ((69.9242474, 0.2038), (71.9220758, 0.2731), (72.9234589, 0.0776), (73.9211778, 0.3672), (75.9214026, 0.0783)),
    "Kr": ((77.9203648, 0.00355), (79.916379, 0.02286), (81.9134836, 0.11593), (82.914136, 0.115), (83.911507, 0.56987), (85.91061073, 0.17279)),
    "Rb": ((84.911789738, 0.7217), (86.909180527, 0.2783)),
    "Sr": ((83.913425, 0.0056), (85.9092602, 0.0986), (86.9088771, 0.07), (87.9056121, 0.8258)),
    "Y": ((88.9058483, 1.0),),
    "Zr": ((89.9047044, 0.5145), (90.9056458, 0.1122), (91.9050408, 0.1715), (93.9063152, 0.1738), (95.9082734, 0.028)),
    "Nb": ((92.9063781, 1.0),),
    "Mo": ((91.906811, 0.1477), (93.9050883, 0.0923), (94.9058421, 0.159), (95.9046795, 0.1668), (96.9060215, 0.0956), (97.9054082, 0.2419), (99.907477, 0.0967)),
    "Ru": ((95.907598, 0.0554), (97.905287, 0.0187), (98.9059393, 0.1276), (99.9042195, 0.126), (100.9055821, 0.1706), (101.9043493, 0.3155), (103.905433, 0.1862)),
    "Rh": ((102.905504, 1.0),),
    "Pd": ((101.905609, 0.0102), (103.904036, 0.1114), (104.905085, 0.2233), (105.903486, 0.2733), (107.903892, 0.2646), (109.905153, 0.1172)),
    "Ag": ((106.905097, 0.51839), (108.904752, 0.48161)),
    "Cd": ((105.906459, 0.0125), (107.904184, 0.0089), (109.9030021, 0.1249), (110.9041781, 0.128), (111.9027578, 0.2413), (112.9044017, 0.1222), (113.9033585, 0.2873), (115.904756, 0.0749)),
    "In": ((112.904058, 0.0429), (114.903878, 0.9571)),
    "Sn": ((111.904818, 0.0097), (113.902779, 0.0066), (114.903342, 0.0034), (115.901741, 0.1454), (116.902952, 0.0768), (117.901603, 0.2422), (118.903308, 0.0859), (119.9021947, 0.3258), (121.903439, 0.0463), (123.9052739, 0.0579)),
    "Sb": ((120.9038157, 0.5721), (122.904214, 0.4279)),
    "Te": ((119.90402, 0.0009), (121.9030439, 0.0255), (122.90427, 0.0089), (123.9028179, 0.0474), (124.9044307, 0.0707), (125.9033117, 0.1884), (127.9044631, 0.3174), (129.9062244, 0.3408)),
    "Xe": ((123.905893, 0.000952), (125.904274, 0.00089), (127.9035313, 0.019102), (128.9047794, 0.264006), (129.903508, 0.04071), (130.9050824, 0.212324), (131.9041535, 0.269086), (133.9053945, 0.104357), (135.907219, 0.088573)),
    "Cs": ((132.905451933, 1.0),),
    "Ba": ((129.9063208, 0.00106), (131.9050613, 0.00101), (133.9045084, 0.02417), (134.9056886, 0.06592), (135.9045759, 0.07854), (136.9058274, 0.11232), (137.9052472, 0.71698)),
    "La": ((137.907112, 0.0009), (138.9063533, 0.9991)),
    "Ce": ((135.907172, 0.00185), (137.905991, 0.00251), (139.9054387, 0.8845), (141.909244, 0.11114)),
    "Pr": ((140.9076528, 1.0),),
    "Nd": ((141.9077233, 0.272), (142.9098143, 0.122), (143.9100873, 0.238), (144.9125736, 0.083), (145.9131169, 0.172), (147.916893, 0.057), (149.920891, 0.056)),
    "Sm": ((143.911999, 0.0307), (146.9148979, 0.1499), (147.9148227, 0.1124), (148.9171847, 0.1382), (149.9172755, 0.0738), (151.9197324, 0.2675), (153.9222093, 0.2275)),
    "Eu": ((150.9198502, 0.4781), (152.9212303, 0.5219)),
    "Gd": ((151.919791, 0.002), (153.9208656, 0.0218), (154.922622, 0.148), (155.9221227, 0.2047), (156.9239601, 0.1565), (157.9241039, 0.2484), (159.9270541, 0.2186)),
    "Tb": ((158.9253468, 1.0),),
    "Dy": ((155.924283, 0.00056), (157.924409, 0.00095), (159.9251975, 0.02329), (160.9269334, 0.18889), (161.9267984, 0.25475), (162.9287312, 0.24896), (163.9291748, 0.2826)),
    "Ho": ((164.9303221, 1.0),),
    "Er": ((161.928778, 0.00139), (163.9292, 0.01601), (165.9302931, 0.33503), (166.9320482, 0.22869), (167.9323702, 0.26978), (169.935464, 0.1491)),
    "Tm": ((168.9342133, 1.0),),
    "Yb": ((167.933897, 0.0013), (169.9347618, 0.0304), (170.9363258, 0.1428), (171.9363815, 0.2183), (172.9382108, 0.1613), (173.9388621, 0.3183), (175.9425717, 0.1276)),
    "Lu": ((174.9407718, 0.9741), (175.9426863, 0.0259)),
    "Hf": ((173.940046, 0.0016), (175.9414086, 0.0526), (176.9432207, 0.186), (177.9436988, 0.2728), (178.9458161, 0.1362), (179.94655, 0.3508)),
    "Ta": ((179.9474648, 0.00012), (180.9479958, 0.99988)),
    "W": ((179.946704, 0.0012), (181.9482042, 0.265), (182.950223, 0.1431), (183.9509312, 0.3064), (185.9543641, 0.2843)),
    "Re": ((184.952955, 0.374), (186.9557531, 0.626)),
    "Os": ((183.9524891, 0.0002), (185.9538382, 0.0159), (186.9557505, 0.0196), (187.9558382, 0.1324), (188.9581475, 0.1615), (189.958447, 0.2626), (191.9614807, 0.4078)),
    "Ir": ((190.960594, 0.373), (192.9629264, 0.627)),
    "Pt": ((189.959932, 0.00014), (191.961038, 0.00782), (193.9626803, 0.32967), (194.9647911, 0.33832), (195.9649515, 0.25242), (197.967893, 0.07163)),
    "Hg": ((195.965833, 0.0015), (197.966769, 0.0997), (198.9682799, 0.1687), (199.968326, 0.231), (200.9703023, 0.1318), (201.970643, 0.2986), (203.9734939, 0.0687)),
    "Tl": ((202.9723442, 0.2952), (204.9744275, 0.7048)),
    "Pb": ((203.9730436, 0.014), (205.9744653, 0.241), (206.9758969, 0.221), (207.9766521, 0.524)),
    "Bi": ((208.9803987, 1.0),),
    "Th": ((232.0380553, 1.0),),
    "U": ((234.0409521, 5.4e-05), (235.0439299, 0.007204), (238.0507882, 0.992742)),
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
