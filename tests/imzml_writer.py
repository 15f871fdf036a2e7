"""Tiny imzML 1.1 writer for test fixtures (our own synthetic files; no reference data).

Writes continuous (one shared m/z array) or processed (per-spectrum arrays) imzML with 32-bit float
m/z and intensity arrays in an external .ibd, the layout sm_distributed_amd.imzml.read_imzml parses.
"""
from __future__ import annotations

import os
import uuid

import numpy as np

_HEAD = """<?xml version="1.0" encoding="ISO-8859-1"?>
<mzML xmlns="http://psi.hupo.org/ms/mzml" version="1.1">
  <cvList count="3">
    <cv id="MS" fullName="Proteomics Standards Initiative Mass Spectrometry Ontology" version="1.3.1" URI="http://psi.hupo.org/ms/mzml"/>
    <cv id="UO" fullName="Unit Ontology" version="1.15" URI="http://obo.cvs.sourceforge.net/obo/obo/ontology/phenotype/unit.obo"/>
    <cv id="IMS" fullName="Imaging MS Ontology" version="0.9.1" URI="http://www.maldi-msi.org/download/imzml/imagingMS.obo"/>
  </cvList>
  <fileDescription>
    <fileContent>
      <cvParam cvRef="MS" accession="MS:1000579" name="MS1 spectrum" value=""/>
      <cvParam cvRef="IMS" accession="IMS:1000080" name="universally unique identifier" value="{uuid}"/>
      <cvParam cvRef="IMS" accession="{mode_acc}" name="{mode}" value=""/>
    </fileContent>
  </fileDescription>
  <referenceableParamGroupList count="2">
    <referenceableParamGroup id="mzArray">
      <cvParam cvRef="MS" accession="MS:1000576" name="no compression" value=""/>
      <cvParam cvRef="MS" accession="MS:1000514" name="m/z array" value=""/>
      <cvParam cvRef="IMS" accession="IMS:1000101" name="external data" value="true"/>
      <cvParam cvRef="MS" accession="MS:1000521" name="32-bit float" value=""/>
    </referenceableParamGroup>
    <referenceableParamGroup id="intensityArray">
      <cvParam cvRef="MS" accession="MS:1000576" name="no compression" value=""/>
      <cvParam cvRef="MS" accession="MS:1000515" name="intensity array" value=""/>
      <cvParam cvRef="IMS" accession="IMS:1000101" name="external data" value="true"/>
      <cvParam cvRef="MS" accession="MS:1000521" name="32-bit float" value=""/>
    </referenceableParamGroup>
  </referenceableParamGroupList>
  <run id="run0">
    <spectrumList count="{n}">
"""

_SPEC = """      <spectrum id="Scan={i1}" defaultArrayLength="0" index="{i}">
        <scanList count="1">
          <scan>
            <cvParam cvRef="IMS" accession="IMS:1000050" name="position x" value="{x}"/>
            <cvParam cvRef="IMS" accession="IMS:1000051" name="position y" value="{y}"/>
          </scan>
        </scanList>
        <binaryDataArrayList count="2">
          <binaryDataArray encodedLength="0">
            <referenceableParamGroupRef ref="mzArray"/>
            <cvParam cvRef="IMS" accession="IMS:1000103" name="external array length" value="{ml}"/>
            <cvParam cvRef="IMS" accession="IMS:1000102" name="external offset" value="{mo}"/>
            <cvParam cvRef="IMS" accession="IMS:1000104" name="external encoded length" value="{mb}"/>
            <binary/>
          </binaryDataArray>
          <binaryDataArray encodedLength="0">
            <referenceableParamGroupRef ref="intensityArray"/>
            <cvParam cvRef="IMS" accession="IMS:1000103" name="external array length" value="{il}"/>
            <cvParam cvRef="IMS" accession="IMS:1000102" name="external offset" value="{io}"/>
            <cvParam cvRef="IMS" accession="IMS:1000104" name="external encoded length" value="{ib}"/>
            <binary/>
          </binaryDataArray>
        </binaryDataArrayList>
      </spectrum>
"""


def write_imzml(path, spectra, continuous=True):
    """spectra: SpectraSet-like (sp_off, mz f32, ints f32, coords).  Writes path and path.ibd."""
    ibd = os.path.splitext(path)[0] + ".ibd"
    u = uuid.UUID(int=12345)
    parts = [u.bytes]
    pos = 16
    entries = []
    shared = None
    for i in range(len(spectra.sp_off) - 1):
        a, b = spectra.sp_off[i], spectra.sp_off[i + 1]
        mz = np.ascontiguousarray(spectra.mz[a:b], np.float32)
        it = np.ascontiguousarray(spectra.ints[a:b], np.float32)
        if continuous and shared is not None:
            mo = shared
        else:
            mo = pos
            parts.append(mz.tobytes())
            pos += mz.nbytes
            if continuous:
                shared = mo
        io = pos
        parts.append(it.tobytes())
        pos += it.nbytes
        entries.append((mz.size, mo, it.size, io))
    with open(ibd, "wb") as f:
        for p in parts:
            f.write(p)
    mode, acc = ("continuous", "IMS:1000030") if continuous else ("processed", "IMS:1000031")
    with open(path, "w", encoding="iso-8859-1") as f:
        f.write(_HEAD.replace("{uuid}", "{" + str(u) + "}").replace("{mode}", mode).replace("{mode_acc}", acc)
                .replace("{n}", str(len(entries))))
        for i, ((ml, mo, il, io), (x, y)) in enumerate(zip(entries, spectra.coords)):
            f.write(_SPEC.format(i=i, i1=i + 1, x=int(x), y=int(y), ml=ml, mo=mo, mb=ml * 4, il=il, io=io, ib=il * 4))
        f.write("    </spectrumList>\n  </run>\n</mzML>\n")
    return path, ibd
