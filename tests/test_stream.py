"""CPU: streaming ingestion -- the native .ess / FASTA readers behind
svh_reader_* against the reference's own data and the restatement of fasta_to_ess.py.

Pinning: covid-19.ess in the reference is fasta_to_ess.py's output for covid-19.fasta (both
committed there; the FASTA is kept as the fixture tests/golden/covid-19.fasta), so the native FASTA
reader must reproduce read_emit_seq(covid-19.ess) exactly, and so must oracle/fasta_oracle.py.
"""
import os

import numpy as np
import pytest

import spec_viterbi_amd as svh
from spec_viterbi_amd import _lib
from oracle.fasta_oracle import ess_text, fasta_sequences
from tests.conftest import ROOT, ess

FASTA = os.path.join(ROOT, "tests", "golden", "covid-19.fasta")


def same_seqs(a, b):
    return len(a) == len(b) and all(np.array_equal(np.asarray(x, np.uint64), np.asarray(y, np.uint64))
                                    for x, y in zip(a, b))


def test_fasta_fixture_reproduces_reference_ess():
    ref = svh.read_emit_seq(ess("covid-19.ess"))
    assert len(ref) == 16
    assert same_seqs(svh.read_sequences(FASTA), ref)                       # native reader
    assert same_seqs(fasta_sequences(open(FASTA).read()), ref)              # restatement


def test_oracle_ess_text_roundtrip(tmp_path):
    seqs = fasta_sequences(open(FASTA).read())
    p = tmp_path / "c.ess"
    p.write_text(ess_text(seqs))
    assert same_seqs(svh.read_emit_seq(str(p)), seqs)


@pytest.mark.parametrize("name", ["emit_3_3500_20.ess", "emit_50_3500_20.ess", "emit_3_7000_20.ess", "covid-19.ess"])
@pytest.mark.parametrize("max_seqs,max_symbols", [(4096, 1 << 22), (1, 1 << 22), (3, 5000), (7, 1)])
def test_ess_streaming_matches_read_emit_seq(name, max_seqs, max_symbols):
    ref = svh.read_emit_seq(ess(name))
    got, chunks = [], 0
    for offs, syms in svh.SeqReader(ess(name), "ess", max_seqs=max_seqs, max_symbols=max_symbols):
        chunks += 1
        nseq = offs.size - 1
        assert 1 <= nseq <= max_seqs
        assert nseq == 1 or offs[-1] <= max_symbols  # whole sequences; a longer one comes alone
        assert syms.dtype == np.uint8 and offs[0] == 0 and offs[-1] == syms.size
        got.extend(syms[offs[q]:offs[q + 1]] for q in range(nseq))
    assert same_seqs(got, ref)
    assert chunks >= -(-len(ref) // max_seqs)


@pytest.mark.parametrize("text", [
    ">a\nACDEF\nGHIKL\n>b\nMNPQRSTVWYX\n",      # multi-line, every residue, X
    "ACD\n>h\n>h2\nEF\n",                        # residues before any header; header-only record
    "  >x  \n  AC DE \r\n>y\nW\n",               # stripped lines; a space inside one is no residue
    ">only header\n",
    "",
])
def test_fasta_cases_match_restatement(tmp_path, text):
    p = tmp_path / "t.fasta"
    p.write_text(text)
    try:
        want = fasta_sequences(text)
    except (KeyError, IndexError) as e:
        with pytest.raises(_lib.SvhError) as err:
            svh.read_sequences(str(p))
        assert err.value.code == (_lib.SVH_E_RANGE if isinstance(e, KeyError) else _lib.SVH_E_IO)
        return
    assert same_seqs(svh.read_sequences(str(p)), want)


@pytest.mark.parametrize("text,code", [
    (">a\nAC\n\nDE\n", "SVH_E_IO"),     # empty line: the script's IndexError at line[0]
    (">a\nACB\n", "SVH_E_RANGE"),       # B is not in amino2num: the script's KeyError
    (">a\nacd\n", "SVH_E_RANGE"),       # lower case is not either
])
def test_fasta_errors(tmp_path, text, code):
    p = tmp_path / "bad.fasta"
    p.write_text(text)
    with pytest.raises(_lib.SvhError) as err:
        svh.read_sequences(str(p))
    assert err.value.code == getattr(_lib, code)


def test_ess_errors_and_format_detection(tmp_path):
    bad = tmp_path / "bad.ess"
    bad.write_text("2\n0 2\n1 2\n5 3\n1 1\n")  # second sequence numbered 5 (data_reader.cpp:112-119)
    with pytest.raises(_lib.SvhError) as err:
        svh.read_sequences(str(bad))
    assert err.value.code == _lib.SVH_E_IO
    big = tmp_path / "big.ess"
    big.write_text("1\n0 2\n1 300\n")  # symbols are uint8 on the device
    with pytest.raises(_lib.SvhError) as err:
        svh.read_sequences(str(big))
    assert err.value.code == _lib.SVH_E_RANGE
    with pytest.raises(_lib.SvhError) as err:
        svh.read_sequences(str(tmp_path / "missing.ess"))
    assert err.value.code == _lib.SVH_E_IO
    # AUTO without a known extension: by content
    a = tmp_path / "seqs.txt"
    a.write_text(open(FASTA).read())
    b = tmp_path / "seqs2.txt"
    b.write_text(open(ess("covid-19.ess")).read())
    assert same_seqs(svh.read_sequences(str(a)), svh.read_sequences(str(b)))
