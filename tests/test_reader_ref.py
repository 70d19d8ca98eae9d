"""CPU: the engine's reader vs the REFERENCE reader compiled from its own sources.

oracle/_ref/ref_reader_dump is built by `make ref` from the reference's
Viterbi_impl/data_reader.cpp (oracle/ref.mk).  Every .chmm / .ess must parse to identical bits.
"""
import glob
import os
import struct
import subprocess

import numpy as np
import pytest

import spec_viterbi_amd as svh
from tests.conftest import DATA, ROOT

REF = os.path.join(ROOT, "oracle", "_ref", "ref_reader_dump")
pytestmark = pytest.mark.skipif(not os.path.exists(REF), reason="oracle/_ref not built (no reference checkout)")


def f2hex(x):
    return struct.pack(">f", float(x)).hex()


def ours_chmm(path):
    h = svh.read_HMM(path)
    out = [str(h.states_num), str(h.emit_num), str(h.start_probabilities.size), str(h.trans_probs.size)]
    for c, v in zip(h.start_probabilities_cols, h.start_probabilities):
        out += [str(int(c)), f2hex(v)]
    out += [f2hex(x) for x in h.emissions.ravel()]
    for s, d, p in zip(h.trans_rows, h.trans_cols, h.trans_probs):
        out += [str(int(s)), str(int(d)), f2hex(p)]
    return out


def ours_ess(path):
    s = svh.read_emit_seq(path)
    out = [str(len(s))]
    for q in s:
        out.append(str(q.size))
        out += [str(int(x)) for x in q]
    return out


CHMMS = sorted(glob.glob(os.path.join(DATA, "chmm_files", "*.chmm")) +
               glob.glob(os.path.join(DATA, "chmm_files", "test_chmms", "*.chmm")))
ESS = sorted(glob.glob(os.path.join(DATA, "ess_files", "*.ess")) +
             glob.glob(os.path.join(DATA, "ess_files", "test_sequences", "*.ess")))


@pytest.mark.parametrize("path", CHMMS, ids=os.path.basename)
def test_chmm_bits_match_reference_reader(path):
    ref = subprocess.run([REF, "chmm", path], capture_output=True, text=True, check=True).stdout.split()
    assert ours_chmm(path) == ref


@pytest.mark.parametrize("path", ESS, ids=os.path.basename)
def test_ess_matches_reference_reader(path):
    ref = subprocess.run([REF, "ess", path], capture_output=True, text=True, check=True).stdout.split()
    assert ours_ess(path) == ref
