"""Minimal imzML/ibd reader: feeds the device layout without the text round trip.

Replaces the ingest path imzml_txt_converter.py:87-140 (pyimzML parse -> ``idx|mzs|ints`` text lines ->
Dataset.txt_to_spectrum_non_cum, dataset.py:106-108).  Supports continuous and processed imzML with
uncompressed 32/64-bit float or 32/64-bit int arrays in the external .ibd file.  Coordinates are the
1-based (x, y) of each spectrum in file order; the pixel map and dims follow dataset.py:52-85.
pyimzML itself is not in this image: this is our own reader of the published imzML 1.1 layout.
"""
from __future__ import annotations

import os
import xml.etree.ElementTree as ET

import numpy as np

from .dataset import to_f32
from .synthetic import SpectraSet

_DTYPES = {"MS:1000521": np.float32, "MS:1000523": np.float64, "IMS:1000141": np.int32, "IMS:1000142": np.int64,
           "MS:1000519": np.int32, "MS:1000522": np.int64}


def _strip(tag):
    return tag.split("}", 1)[1] if "}" in tag else tag


def read_imzml(imzml_path: str, ibd_path: str | None = None) -> SpectraSet:
    ibd_path = ibd_path or os.path.splitext(imzml_path)[0] + ".ibd"
    tree = ET.parse(imzml_path)
    root = tree.getroot()
    groups = {}
    for g in root.iter():
        if _strip(g.tag) == "referenceableParamGroup":
            groups[g.get("id")] = [c.get("accession") for c in g if _strip(c.tag) == "cvParam"]

    def params(el):
        acc = {}
        for c in el.iter():
            t = _strip(c.tag)
            if t == "cvParam":
                acc[c.get("accession")] = c.get("value")
            elif t == "referenceableParamGroupRef":
                for a in groups.get(c.get("ref"), []):
                    acc.setdefault(a, "")
        return acc

    coords, arrays = [], []
    for sp in root.iter():
        if _strip(sp.tag) != "spectrum":
            continue
        p = params(sp)
        x, y = int(p["IMS:1000050"]), int(p["IMS:1000051"])
        coords.append((x, y))
        mz_a = int_a = None
        for bda in sp.iter():
            if _strip(bda.tag) != "binaryDataArray":
                continue
            bp = params(bda)
            dt = next((v for k, v in _DTYPES.items() if k in bp), np.float32)
            desc = (int(bp["IMS:1000102"]), int(bp["IMS:1000103"]), dt)
            if "MS:1000514" in bp:
                mz_a = desc
            elif "MS:1000515" in bp:
                int_a = desc
        arrays.append((mz_a, int_a))
    with open(ibd_path, "rb") as f:
        buf = f.read()
    off = np.zeros(len(arrays) + 1, np.int64)
    mzs, its = [], []
    for i, ((mo, ml, mdt), (io, il, idt)) in enumerate(arrays):
        mz = to_f32(np.frombuffer(buf, dtype=mdt, count=ml, offset=mo), "m/z")
        it = to_f32(np.frombuffer(buf, dtype=idt, count=il, offset=io), "intensity")
        mzs.append(mz)
        its.append(it)
        off[i + 1] = off[i] + ml
    return SpectraSet(sp_off=off, mz=np.concatenate(mzs) if mzs else np.zeros(0, np.float32),
                      ints=np.concatenate(its) if its else np.zeros(0, np.float32), coords=np.asarray(coords))
