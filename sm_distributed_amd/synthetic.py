"""Seeded synthetic datasets and ion tables.

The reference's real inputs (HMDB, the spheroid imzML, cpyMSpec isotope patterns) are not available
offline, so benchmarks and parity tests run on synthetic data of the documented shape:

* spectra: ``nrows x ncols`` grid, spectrum index row-major, ``P ~ Poisson(peaks_per_spectrum)``
  centroids per spectrum, m/z ~ U[mz_min, mz_max) (f64 -> f32, sorted per spectrum as a centroided
  imzML spectrum is), intensities ~ LogNormal(6, 1.5) -> f32;
* ion table: ``n_sf`` synthetic formulas with monoisotopic mass ~ U[150, 900], K ~ U{4..6} isotope
  peaks spaced 1.003355 Da, intensities ``100*exp(-a*k)``; target adducts +H/+Na/+K and, per
  ``fdr.py:27-31``, ``decoy_sample_size`` decoy adducts drawn per (sf, target adduct) from the 80
  element adducts (seeded, so the target/decoy table is reproducible);
* planted signal: a fraction of target ions get all K peaks (m/z jittered by N(0, 0.5 ppm)) in the
  pixels of a random Gaussian blob with intensity proportional to the theoretical pattern.

Two generators share this recipe: ``make_dataset_np`` (numpy, host; small parity cases, the oracle
consumes exactly these arrays) and ``make_dataset_torch`` (torch on the GPU; the 5e8-point bench
dataset, generated in seconds directly in HBM).  Their random streams differ; each is seeded.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

# fdr.py:8 -- the decoy adduct candidates
DECOY_ADDUCTS = ['+He', '+Li', '+Be', '+B', '+C', '+N', '+O', '+F', '+Ne', '+Mg', '+Al', '+Si', '+P',
                 '+S', '+Cl', '+Ar', '+Ca', '+Sc', '+Ti', '+V', '+Cr', '+Mn', '+Fe', '+Co', '+Ni', '+Cu',
                 '+Zn', '+Ga', '+Ge', '+As', '+Se', '+Br', '+Kr', '+Rb', '+Sr', '+Y', '+Zr', '+Nb', '+Mo',
                 '+Ru', '+Rh', '+Pd', '+Ag', '+Cd', '+In', '+Sn', '+Sb', '+Te', '+I', '+Xe', '+Cs', '+Ba',
                 '+La', '+Ce', '+Pr', '+Nd', '+Sm', '+Eu', '+Gd', '+Tb', '+Dy', '+Ho', '+Ir', '+Th', '+Pt',
                 '+Os', '+Yb', '+Lu', '+Bi', '+Pb', '+Re', '+Tl', '+Tm', '+U', '+W', '+Au', '+Er', '+Hf',
                 '+Hg', '+Ta']

# monoisotopic masses of the most abundant isotope (synthetic adduct shifts)
ELEMENT_MASS = {
    'H': 1.007825, 'Na': 22.989770, 'K': 38.963707, 'He': 4.002603, 'Li': 7.016004, 'Be': 9.012182,
    'B': 11.009305, 'C': 12.0, 'N': 14.003074, 'O': 15.994915, 'F': 18.998403, 'Ne': 19.992440,
    'Mg': 23.985042, 'Al': 26.981539, 'Si': 27.976927, 'P': 30.973762, 'S': 31.972071,
    'Cl': 34.968853, 'Ar': 39.962383, 'Ca': 39.962591, 'Sc': 44.955912, 'Ti': 47.947946,
    'V': 50.943960, 'Cr': 51.940508, 'Mn': 54.938045, 'Fe': 55.934938, 'Co': 58.933195,
    'Ni': 57.935343, 'Cu': 62.929598, 'Zn': 63.929142, 'Ga': 68.925574, 'Ge': 73.921178,
    'As': 74.921597, 'Se': 79.916521, 'Br': 78.918337, 'Kr': 83.911507, 'Rb': 84.911790,
    'Sr': 87.905612, 'Y': 88.905848, 'Zr': 89.904704, 'Nb': 92.906378, 'Mo': 97.905408,
    'Ru': 101.904349, 'Rh': 102.905504, 'Pd': 105.903486, 'Ag': 106.905097, 'Cd': 113.903359,
    'In': 114.903878, 'Sn': 119.902195, 'Sb': 120.903816, 'Te': 129.906224, 'I': 126.904473,
    'Xe': 131.904154, 'Cs': 132.905452, 'Ba': 137.905247, 'La': 138.906353, 'Ce': 139.905439,
    'Pr': 140.907653, 'Nd': 141.907723, 'Sm': 151.919732, 'Eu': 152.921230, 'Gd': 157.924104,
    'Tb': 158.925347, 'Dy': 163.929175, 'Ho': 164.930322, 'Ir': 192.962926, 'Th': 232.038055,
    'Pt': 194.964791, 'Os': 191.961481, 'Yb': 173.938862, 'Lu': 174.940772, 'Bi': 208.980399,
    'Pb': 207.976652, 'Re': 186.955753, 'Tl': 204.974428, 'Tm': 168.934213, 'U': 238.050788,
    'W': 183.950931, 'Au': 196.966569, 'Er': 165.930293, 'Hf': 179.946550, 'Hg': 201.970643,
    'Ta': 180.947996,
}
ELECTRON_MASS = 0.00054858
ISOTOPE_SPACING = 1.003355
TARGET_ADDUCTS = ('+H', '+Na', '+K')


# BASELINE config 5: 6 target adducts in both polarities (a positive-mode and a negative-mode search over the same
# molecule table); the charge sign follows the polarity (isocalc_wrapper.py:28-32)
TARGET_ADDUCTS_POS = ('+H', '+Na', '+K')
TARGET_ADDUCTS_NEG = ('-H', '+Cl', '+Br')


def adduct_shift(adduct: str, charge: int = 1) -> float:
    """m/z shift of ``sf + adduct`` at charge +-1: the adduct adds ('+X') or removes ('-X') element X, and the
    ion carries ``charge`` missing electrons (complete_isodist(..., charge), isocalc_wrapper.py:28-40: m/z =
    (M - z*m_e) / |z|), so a negative ion is one electron mass heavier than its neutral."""
    if charge not in (1, -1):
        raise ValueError("synthetic ion tables are singly charged")
    sign = 1.0 if adduct[0] == '+' else -1.0
    return sign * ELEMENT_MASS[adduct[1:]] - charge * ELECTRON_MASS


@dataclass
class FormulaSet:
    """Synthetic sum formulas (CHNOPS compositions): ``sf`` strings, monoisotopic neutral ``mass`` and element
    ``counts`` [n_sf, len(FORMULA_ELEMENTS)], so negative adducts can be vetted as theor_peaks_gen.py:46-51 does
    ('-X' needs element X in the formula)."""
    sf: np.ndarray
    mass: np.ndarray
    counts: np.ndarray

    def has_element(self, el: str) -> np.ndarray:
        if el not in FORMULA_ELEMENTS:
            return np.zeros(len(self.sf), dtype=bool)
        return self.counts[:, FORMULA_ELEMENTS.index(el)] > 0


FORMULA_ELEMENTS = ('C', 'H', 'N', 'O', 'P', 'S')


def make_formulas(n_sf: int, seed: int = 43, mass_range=(150.0, 900.0), no_h_fraction: float = 0.01) -> FormulaSet:
    """``n_sf`` distinct organic compositions (unique sum formulas, as the reference's agg_formula table) with
    monoisotopic mass in ``mass_range``: C from the mass, H from a drawn degree of unsaturation (H = 2C + 2 + N -
    2*DBE), N/P/S sparse, O filling the mass; ``no_h_fraction`` of them carry no hydrogen, so the '-H' adduct is
    vetted out for those formulas as the reference does."""
    rng = np.random.default_rng(seed)
    el_mass = np.array([ELEMENT_MASS[e] for e in FORMULA_ELEMENTS])
    rows, seen = [], set()
    while len(rows) < n_sf:
        k = 2 * (n_sf - len(rows)) + 16
        m = rng.uniform(mass_range[0], mass_range[1], k)
        c = np.maximum(1, np.round(m * rng.uniform(0.035, 0.06, k))).astype(np.int64)
        n = rng.poisson(0.8, k)
        ph = (rng.random(k) < 0.05).astype(np.int64)
        su = (rng.random(k) < 0.06).astype(np.int64)
        dbe = np.floor(rng.random(k) * (c // 2 + 1)).astype(np.int64)
        h = 2 * c + 2 + n - 2 * dbe
        h = np.where(rng.random(k) < no_h_fraction, 0, h)
        rest = m - (c * el_mass[0] + h * el_mass[1] + n * el_mass[2] + ph * el_mass[4] + su * el_mass[5])
        o = np.round(rest / el_mass[3]).astype(np.int64)
        cnt = np.stack([c, h, n, o, ph, su], axis=1)
        mass = cnt @ el_mass
        ok = (h >= 0) & (o >= 0) & (mass >= mass_range[0]) & (mass <= mass_range[1])
        for r in cnt[ok].tolist():
            t = tuple(r)
            if t not in seen and len(rows) < n_sf:
                seen.add(t)
                rows.append(r)
    counts = np.array(rows, dtype=np.int64).reshape(n_sf, len(FORMULA_ELEMENTS))
    mass = counts @ el_mass

    def name(row):
        return ''.join(e + (str(k) if k > 1 else '') for e, k in zip(FORMULA_ELEMENTS, row) if k > 0)
    sf = np.array([name(r) for r in counts.tolist()], dtype=object)
    return FormulaSet(sf=sf, mass=mass, counts=counts)


@dataclass
class IonTable:
    """Per-ion theoretical peaks, the shape ``FormulasSegm`` exposes (formulas_segm.py:56-69).

    ``sf_ids``/``adducts`` identify each ion; ``win_off`` (n_ion+1) delimits its windows in
    ``peak_mz``/``peak_int`` (ion-major, peak_i order).  ``td_df`` is the target/decoy table
    (columns sf_id, ta, da) as ``FDR.decoy_adduct_selection`` builds it (fdr.py:42-48).
    """
    sf_ids: np.ndarray
    adducts: np.ndarray
    win_off: np.ndarray
    peak_mz: np.ndarray
    peak_int: np.ndarray
    target_adducts: tuple = TARGET_ADDUCTS
    decoy_sample_size: int = 20
    td: tuple = field(default=None)   # (sf_id, ta, da) arrays
    is_target: np.ndarray = None      # bool per ion (None: adduct in target_adducts)
    charge: np.ndarray = None         # +-1 per ion (None: +1)
    sf_names: np.ndarray = None       # sum formula string per sf_id - sf_id_offset (FormulaSet tables)

    def target_mask(self):
        if self.is_target is not None:
            return self.is_target
        return np.isin(self.adducts, list(self.target_adducts))

    @property
    def n_ions(self):
        return len(self.sf_ids)

    @property
    def n_windows(self):
        return int(self.win_off[-1])

    def sf_df(self):
        """(sf_id, adduct, centr_mzs, centr_ints) rows sorted by (sf_id, adduct) -- FormulasSegm.sf_df."""
        import pandas as pd
        mzs = [self.peak_mz[a:b].tolist() for a, b in zip(self.win_off[:-1], self.win_off[1:])]
        ints = [self.peak_int[a:b].tolist() for a, b in zip(self.win_off[:-1], self.win_off[1:])]
        df = pd.DataFrame({'sf_id': self.sf_ids, 'adduct': self.adducts, 'centr_mzs': mzs, 'centr_ints': ints})
        return df.sort_values(['sf_id', 'adduct']).reset_index(drop=True)

    def td_df(self):
        import pandas as pd
        sf, ta, da = self.td
        return pd.DataFrame({'sf_id': sf, 'ta': ta, 'da': da})


def make_ion_table(n_sf: int, seed: int = 43, decoy_seed: int = 44, target_adducts=TARGET_ADDUCTS,
                   decoy_sample_size: int = 20, mass_range=(150.0, 900.0), k_range=(4, 6),
                   sf_id_offset: int = 0, formulas: FormulaSet | None = None, charge: int = 1) -> IonTable:
    """Ion table of one search: ``n_sf`` formulas x target adducts + distinct decoys.  ``formulas`` (a
    FormulaSet) gives the neutral masses and compositions (else masses are drawn uniformly and every adduct is
    valid); ``charge`` +-1 is the polarity's (isocalc_wrapper.py:28-32).  A target ion whose '-X' adduct removes
    an element the formula lacks is not generated (theor_peaks_gen.py:46-51: no theoretical peaks, so no row in
    sf_df), while its decoy draws stay in the target/decoy table as FDR.decoy_adduct_selection makes them."""
    rng = np.random.default_rng(seed)
    mass = rng.uniform(mass_range[0], mass_range[1], n_sf)
    n_peaks = rng.integers(k_range[0], k_range[1] + 1, n_sf)
    decay = rng.uniform(0.5, 2.5, n_sf)
    if formulas is not None:
        assert len(formulas.mass) == n_sf
        mass = formulas.mass
    sf_ids = np.arange(n_sf, dtype=np.int64) + sf_id_offset

    # fdr.py:27-31 / :42-48: per (sf, target adduct) draw decoy_sample_size decoys without replacement
    cand = sorted(set(DECOY_ADDUCTS) - set(target_adducts))
    drng = np.random.default_rng(decoy_seed)
    n_ta = len(target_adducts)
    draws = np.argsort(drng.random((n_sf * n_ta, len(cand))), axis=1)[:, :decoy_sample_size]
    td_sf = np.repeat(sf_ids, n_ta * decoy_sample_size)
    td_ta = np.tile(np.repeat(np.array(target_adducts, dtype=object), decoy_sample_size), n_sf)
    cand_arr = np.array(cand, dtype=object)
    td_da = cand_arr[draws.reshape(-1)]

    # ion set = targets + DISTINCT decoys per sf (formulas_segm.py:14-20 SELECT DISTINCT)
    used = np.zeros((n_sf, len(cand)), dtype=bool)
    used[np.repeat(np.arange(n_sf), n_ta * decoy_sample_size), draws.reshape(-1)] = True
    t_sf = np.repeat(np.arange(n_sf), n_ta)
    t_add = np.tile(np.array(target_adducts, dtype=object), n_sf)
    if formulas is not None:  # theor_peaks_gen.py:46-51: '-X' needs X in the formula
        valid = np.ones(t_sf.size, dtype=bool)
        for j, a in enumerate(target_adducts):
            if a.startswith('-'):
                valid[j::n_ta] = formulas.has_element(a[1:])
        t_sf, t_add = t_sf[valid], t_add[valid]
    ion_sf_idx = [t_sf]
    ion_add = [t_add]
    dsf, dc = np.nonzero(used)
    ion_sf_idx.append(dsf)
    ion_add.append(cand_arr[dc])
    is_tgt = np.concatenate([np.ones(t_sf.size, bool), np.zeros(dsf.size, bool)])
    ion_sf_idx = np.concatenate(ion_sf_idx)
    ion_add = np.concatenate(ion_add)
    order = np.lexsort((ion_add.astype(str), ion_sf_idx))
    ion_sf_idx, ion_add, is_tgt = ion_sf_idx[order], ion_add[order], is_tgt[order]

    shifts = {a: adduct_shift(a, charge) for a in set(ion_add.tolist())}
    ion_mz0 = mass[ion_sf_idx] + np.array([shifts[a] for a in ion_add])
    K = n_peaks[ion_sf_idx]
    win_off = np.zeros(len(K) + 1, dtype=np.int64)
    np.cumsum(K, out=win_off[1:])
    within = np.arange(win_off[-1]) - np.repeat(win_off[:-1], K)
    owner = np.repeat(np.arange(len(K)), K)
    peak_mz = ion_mz0[owner] + within * ISOTOPE_SPACING
    peak_int = 100.0 * np.exp(-decay[ion_sf_idx][owner] * within)
    # theor_peaks stores %.6f text (theor_peaks_gen.py:76-84)
    peak_mz = np.round(peak_mz, 6)
    peak_int = np.round(peak_int, 6)
    return IonTable(sf_ids=sf_ids[ion_sf_idx], adducts=ion_add, win_off=win_off, peak_mz=peak_mz,
                    peak_int=peak_int, target_adducts=tuple(target_adducts),
                    decoy_sample_size=decoy_sample_size, td=(td_sf, td_ta, td_da),
                    is_target=is_tgt if formulas is not None else None,
                    charge=np.full(len(ion_add), charge, np.int8) if charge != 1 else None,
                    sf_names=formulas.sf if formulas is not None else None)


def concat_ion_tables(tables) -> IonTable:
    """One ion table from several searches over disjoint sf_id ranges (e.g. both polarities)."""
    off = [np.zeros(1, np.int64)]
    base = 0
    for t in tables:
        off.append(t.win_off[1:] + base)
        base += int(t.win_off[-1])
    cat = lambda f: np.concatenate([f(t) for t in tables])
    return IonTable(sf_ids=cat(lambda t: t.sf_ids), adducts=cat(lambda t: t.adducts), win_off=np.concatenate(off),
                    peak_mz=cat(lambda t: t.peak_mz), peak_int=cat(lambda t: t.peak_int),
                    target_adducts=tuple(a for t in tables for a in t.target_adducts),
                    decoy_sample_size=tables[0].decoy_sample_size,
                    td=tuple(np.concatenate([t.td[j] for t in tables]) for j in range(3)),
                    is_target=cat(lambda t: t.target_mask()),
                    charge=cat(lambda t: t.charge if t.charge is not None else np.ones(t.n_ions, np.int8)))


def make_ion_table_both_polarities(n_sf: int, seed: int = 43, decoy_seed: int = 44,
                                   pos_adducts=TARGET_ADDUCTS_POS, neg_adducts=TARGET_ADDUCTS_NEG,
                                   decoy_sample_size: int = 20, mass_range=(150.0, 900.0)) -> IonTable:
    """BASELINE config 5's table: the same ``n_sf`` formulas searched in positive mode (sf_id 0..n_sf-1, charge
    +1, ``pos_adducts``) and negative mode (sf_id n_sf..2n_sf-1, charge -1, ``neg_adducts``), each with its own
    decoys (fdr.py:42-48: candidates = DECOY_ADDUCTS minus that search's targets).  The reference runs one
    polarity per dataset config; the two searches' ions are kept apart by sf_id so (sf_id, adduct) stays unique
    (a '+Cl' positive-mode decoy and the '+Cl' negative-mode target are different ions)."""
    fs = make_formulas(n_sf, seed=seed + 1000, mass_range=mass_range)
    pos = make_ion_table(n_sf, seed=seed, decoy_seed=decoy_seed, target_adducts=pos_adducts,
                         decoy_sample_size=decoy_sample_size, formulas=fs, charge=1)
    neg = make_ion_table(n_sf, seed=seed, decoy_seed=decoy_seed + 1, target_adducts=neg_adducts,
                         decoy_sample_size=decoy_sample_size, formulas=fs, charge=-1, sf_id_offset=n_sf)
    out = concat_ion_tables([pos, neg])
    out.sf_names = fs.sf
    return out


@dataclass
class SpectraSet:
    """Host-side dataset: spectra in pixel order plus the reference's pixel map and dims.

    ``sp_off`` (n_sp+1) delimits spectrum i's points in ``mz`` (f32) / ``ints`` (f32);
    ``coords`` are the 1-based (x, y) of each spectrum (imzml_txt_converter.py:120-123), from which
    ``pixel_map``/``dims`` follow exactly as dataset.py:52-85 computes them.
    """
    sp_off: np.ndarray
    mz: np.ndarray
    ints: np.ndarray
    coords: np.ndarray

    @property
    def n_spectra(self):
        return len(self.sp_off) - 1

    @property
    def n_points(self):
        return int(self.sp_off[-1])

    def pixel_map_dims(self):
        return pixel_map_from_coords(self.coords)

    def spectra(self):
        """(sp_id, mz f32[], int f64[]) tuples as Dataset.txt_to_spectrum_non_cum yields (dataset.py:106-108)."""
        for i in range(self.n_spectra):
            a, b = self.sp_off[i], self.sp_off[i + 1]
            yield i, self.mz[a:b], self.ints[a:b].astype(np.float64)


def pixel_map_from_coords(coords):
    """dataset.py:52-85: pixel = (y - min_y) * ncols + (x - min_x); dims = (nrows, ncols)."""
    c = np.asarray(coords, dtype=np.int64)
    mn = c.min(axis=0)
    mx = c.max(axis=0)
    ncols = int(mx[0] - mn[0] + 1)
    nrows = int(mx[1] - mn[1] + 1)
    c = c - mn
    pix = (c[:, 1] * ncols + c[:, 0]).astype(np.int32)
    return pix, (nrows, ncols)


def make_dataset_np(nrows: int, ncols: int, peaks_per_spectrum: float, seed: int = 42,
                    mz_range=(100.0, 1000.0), ions: IonTable | None = None, plant_fraction: float = 0.0,
                    plant_seed: int = 45, blob_sigma=(2.0, 6.0), zero_fraction: float = 0.0) -> SpectraSet:
    rng = np.random.default_rng(seed)
    n_sp = nrows * ncols
    counts = rng.poisson(peaks_per_spectrum, n_sp).astype(np.int64)
    mz = rng.uniform(mz_range[0], mz_range[1], int(counts.sum())).astype(np.float32)
    ints = rng.lognormal(6.0, 1.5, mz.shape[0]).astype(np.float32)
    if zero_fraction > 0:
        ints[rng.random(ints.shape[0]) < zero_fraction] = 0.0
    sp_of = np.repeat(np.arange(n_sp), counts)
    if ions is not None and plant_fraction > 0:
        p_sp, p_mz, p_int = _plant_np(ions, nrows, ncols, plant_fraction, plant_seed, blob_sigma, mz_range)
        sp_of = np.concatenate([sp_of, p_sp])
        mz = np.concatenate([mz, p_mz])
        ints = np.concatenate([ints, p_int])
    # centroided spectra are m/z sorted within each spectrum
    order = np.lexsort((mz, sp_of))
    sp_of, mz, ints = sp_of[order], mz[order], ints[order]
    sp_off = np.zeros(n_sp + 1, dtype=np.int64)
    np.cumsum(np.bincount(sp_of, minlength=n_sp), out=sp_off[1:])
    ys, xs = np.divmod(np.arange(n_sp), ncols)
    coords = np.stack([xs + 1, ys + 1], axis=1)
    return SpectraSet(sp_off=sp_off, mz=mz, ints=ints, coords=coords)


def _plant_np(ions: IonTable, nrows, ncols, fraction, seed, blob_sigma, mz_range):
    rng = np.random.default_rng(seed)
    tgt = np.nonzero(ions.target_mask())[0]
    n_pl = max(1, int(round(fraction * len(tgt)))) if len(tgt) else 0
    chosen = rng.choice(tgt, size=n_pl, replace=False) if n_pl else np.zeros(0, np.int64)
    sp_l, mz_l, in_l = [], [], []
    yy, xx = np.mgrid[0:nrows, 0:ncols]
    for ion in chosen:
        cy, cx = rng.uniform(0, nrows), rng.uniform(0, ncols)
        sig = rng.uniform(*blob_sigma)
        amp = rng.lognormal(8.0, 0.5)
        g = np.exp(-((yy - cy) ** 2 + (xx - cx) ** 2) / (2 * sig * sig))
        sel = rng.random(g.shape) < g
        pix = np.nonzero(sel.ravel())[0]
        a, b = ions.win_off[ion], ions.win_off[ion + 1]
        for k in range(a, b):
            mzk = ions.peak_mz[k]
            if not (mz_range[0] <= mzk < mz_range[1]):
                continue
            jit = mzk * (1.0 + rng.normal(0.0, 0.5e-6, pix.shape[0]))
            sp_l.append(pix)
            mz_l.append(jit.astype(np.float32))
            in_l.append((amp * g.ravel()[pix] * ions.peak_int[k] / 100.0).astype(np.float32))
    if not sp_l:
        return np.zeros(0, np.int64), np.zeros(0, np.float32), np.zeros(0, np.float32)
    return np.concatenate(sp_l), np.concatenate(mz_l), np.concatenate(in_l)


# At or above this many background points (config 5: 1000x1000 px x Poisson(5000) = 5e9) the dataset is
# generated block by block of spectra, straight into the resident arrays: the one-shot recipe below needs a
# global 64-bit key sort whose temporaries alone would exceed HBM.  Smaller datasets (config 3) keep the
# one-shot recipe and its RNG stream, so their contents do not change.
CHUNKED_GEN_POINTS = 1 << 31
CHUNK_POINTS = 1 << 28


def _assemble_chunked(g, counts, n_sp, mz_range, extra_pix, extra_mz, extra_int, device):
    """Spectrum-major (mz f32[N], hits i64[N], sp_off i64[n_sp+1]) built one block of spectra at a time."""
    import torch
    if extra_pix:
        e_pix = torch.cat(extra_pix)
        e_mz = torch.cat(extra_mz)
        e_int = torch.cat(extra_int)
        o = torch.argsort(e_pix, stable=True)
        e_pix, e_mz, e_int = e_pix[o], e_mz[o], e_int[o]
        tot = counts + torch.bincount(e_pix, minlength=n_sp)
    else:
        e_pix = torch.zeros(0, dtype=torch.int64, device=device)
        e_mz = torch.zeros(0, dtype=torch.float32, device=device)
        e_int = torch.zeros(0, dtype=torch.float32, device=device)
        tot = counts
    sp_off = torch.zeros(n_sp + 1, dtype=torch.int64, device=device)
    sp_off[1:] = torch.cumsum(tot, 0)
    n_all = int(sp_off[-1].item())
    mz_out = torch.empty(n_all, dtype=torch.float32, device=device)
    hits_out = torch.empty(n_all, dtype=torch.int64, device=device)
    off_h = sp_off.cpu().numpy()
    bg_h = np.concatenate([[0], np.cumsum(counts.cpu().numpy())])
    s0 = 0
    while s0 < n_sp:
        s1 = int(np.searchsorted(off_h, off_h[s0] + CHUNK_POINTS, side="right")) - 1
        s1 = min(max(s1, s0 + 1), n_sp)
        nb = int(bg_h[s1] - bg_h[s0])
        mz = (torch.rand(nb, generator=g, dtype=torch.float64, device=device) * (mz_range[1] - mz_range[0])
              + mz_range[0]).to(torch.float32)
        ints = torch.exp(torch.randn(nb, generator=g, dtype=torch.float32, device=device) * 1.5 + 6.0)
        pix = torch.repeat_interleave(torch.arange(s0, s1, device=device, dtype=torch.int64), counts[s0:s1])
        if e_pix.numel():
            a, b = torch.searchsorted(e_pix, torch.tensor([s0, s1], device=device, dtype=torch.int64)).tolist()
            if b > a:
                pix = torch.cat([pix, e_pix[a:b]])
                mz = torch.cat([mz, e_mz[a:b]])
                ints = torch.cat([ints, e_int[a:b]])
        key = (pix << 32) | mz.view(torch.int32).to(torch.int64)
        order = torch.sort(key).indices
        del key
        lo, hi = int(off_h[s0]), int(off_h[s1])
        assert hi - lo == order.numel()
        mz_out[lo:hi] = mz[order]
        hits_out[lo:hi] = (pix[order] & 0xFFFFFFFF) | (ints[order].view(torch.int32).to(torch.int64) << 32)
        del mz, ints, pix, order
        s0 = s1
    return mz_out, hits_out, sp_off


def make_dataset_torch(nrows: int, ncols: int, peaks_per_spectrum: float, seed: int = 42, device="cuda",
                       mz_range=(100.0, 1000.0), ions: IonTable | None = None, plant_fraction: float = 0.02,
                       plant_seed: int = 45, blob_sigma=(3.0, 12.0)):
    """Config-3 style dataset generated directly in HBM (same recipe as make_dataset_np, torch RNG).

    Returns ``(mz f32[N], hits int64[N], dims, info)`` in the resident layout (hits = pixel | f32 << 32),
    spectrum-major (dataset order); pixel = spectrum index (row-major grid, dataset.py:52-66).
    """
    import torch
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    n_sp = nrows * ncols
    counts = torch.poisson(torch.full((n_sp,), float(peaks_per_spectrum), device=device, dtype=torch.float32),
                           generator=g).to(torch.int64)
    n = int(counts.sum().item())
    chunked = n >= CHUNKED_GEN_POINTS
    if not chunked:
        mz = (torch.rand(n, generator=g, dtype=torch.float64, device=device) * (mz_range[1] - mz_range[0])
              + mz_range[0]).to(torch.float32)
        ints = torch.exp(torch.randn(n, generator=g, dtype=torch.float32, device=device) * 1.5 + 6.0)
        pix = torch.repeat_interleave(torch.arange(n_sp, device=device, dtype=torch.int64), counts)
    extra_pix, extra_mz, extra_int = [], [], []
    n_planted = 0
    if ions is not None and plant_fraction > 0:
        rng = np.random.default_rng(plant_seed)
        tgt = np.nonzero(ions.target_mask())[0]
        n_pl = max(1, int(round(plant_fraction * len(tgt)))) if len(tgt) else 0
        chosen = rng.choice(tgt, size=n_pl, replace=False) if n_pl else []
        gp = torch.Generator(device=device)
        gp.manual_seed(plant_seed)
        for ion in chosen:
            cy, cx = rng.uniform(0, nrows), rng.uniform(0, ncols)
            sig = rng.uniform(*blob_sigma)
            amp = float(rng.lognormal(8.0, 0.5))
            r0, r1 = max(0, int(cy - 4 * sig)), min(nrows, int(cy + 4 * sig) + 1)
            c0, c1 = max(0, int(cx - 4 * sig)), min(ncols, int(cx + 4 * sig) + 1)
            yy = torch.arange(r0, r1, device=device, dtype=torch.float64)[:, None]
            xx = torch.arange(c0, c1, device=device, dtype=torch.float64)[None, :]
            gauss = torch.exp(-((yy - cy) ** 2 + (xx - cx) ** 2) / (2 * sig * sig))
            sel = torch.rand(gauss.shape, generator=gp, device=device, dtype=torch.float64) < gauss
            rr, cc = torch.nonzero(sel, as_tuple=True)
            if rr.numel() == 0:
                continue
            p = (rr + r0) * ncols + (cc + c0)
            gv = gauss[rr, cc]
            a, b = ions.win_off[ion], ions.win_off[ion + 1]
            for k in range(a, b):
                mzk = float(ions.peak_mz[k])
                if not (mz_range[0] <= mzk < mz_range[1]):
                    continue
                jit = mzk * (1.0 + torch.randn(p.numel(), generator=gp, device=device, dtype=torch.float64) * 0.5e-6)
                extra_pix.append(p)
                extra_mz.append(jit.to(torch.float32))
                extra_int.append((amp * gv * float(ions.peak_int[k]) / 100.0).to(torch.float32))
            n_planted += 1
    if chunked:
        mz, hits, sp_off = _assemble_chunked(g, counts, n_sp, mz_range, extra_pix, extra_mz, extra_int, device)
        info = {"n_points": int(mz.numel()), "n_spectra": n_sp, "n_planted_ions": n_planted,
                "n_planted_points": int(sum(t.numel() for t in extra_mz)), "sp_off": sp_off}
        return mz, hits, (nrows, ncols), info
    if extra_pix:
        pix = torch.cat([pix] + extra_pix)
        mz = torch.cat([mz] + extra_mz)
        ints = torch.cat([ints] + extra_int)
    # dataset order: spectrum-major, each spectrum m/z-sorted (as a centroided imzML spectrum is)
    key = (pix << 32) | mz.view(torch.int32).to(torch.int64)
    order = torch.sort(key).indices
    del key
    pix, mz, ints = pix[order], mz[order], ints[order]
    del order
    counts = torch.bincount(pix, minlength=n_sp)
    sp_off = torch.zeros(n_sp + 1, dtype=torch.int64, device=device)
    sp_off[1:] = torch.cumsum(counts, 0)
    hits = (pix & 0xFFFFFFFF) | (ints.view(torch.int32).to(torch.int64) << 32)
    del pix, ints
    info = {"n_points": int(mz.numel()), "n_spectra": n_sp, "n_planted_ions": n_planted,
            "n_planted_points": int(sum(t.numel() for t in extra_mz)), "sp_off": sp_off}
    return mz, hits, (nrows, ncols), info
