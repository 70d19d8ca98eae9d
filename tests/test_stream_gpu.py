"""GPU: the pipelined file decoder (svh_decode_file) against the oracle and the one-shot path."""
import os

import numpy as np
import pytest

import spec_viterbi_amd as svh
from spec_viterbi_amd import _lib
from oracle import oracle
from oracle.fasta_oracle import ess_text
from tests.conftest import ROOT, chmm, ess
from tests.helpers import bit_equal, from_hex, load_golden, random_hmm, random_seqs

pytestmark = pytest.mark.gpu
FASTA = os.path.join(ROOT, "tests", "golden", "covid-19.fasta")


@pytest.mark.parametrize("max_seqs,max_symbols", [(3, 1 << 22), (16, 2000), (1, 1)])
def test_decode_fasta_with_paths_vs_oracle(max_seqs, max_symbols):
    """covid-19.fasta -> 2405.chmm: scores, best states and paths of every sequence equal the
    oracle's, whatever the chunking (ragged 38..7096 observations)."""
    hmm = svh.read_HMM(chmm("2405.chmm"))
    model = svh.DeviceModel(hmm)
    scores, best, paths = svh.decode_file(model, FASTA, paths=True, max_seqs=max_seqs, max_symbols=max_symbols)
    seqs = svh.read_sequences(FASTA)
    assert scores.shape == (16, hmm.states_num)
    for q, seq in enumerate(seqs):
        ref, ref_best, ref_path = oracle.decode(hmm, seq)
        assert bit_equal(scores[q], ref), q
        assert best[q] == ref_best, q
        assert np.array_equal(paths[q], ref_path), q


def test_decode_ess_scores_vs_golden_and_one_shot():
    hmm = svh.read_HMM(chmm("2405.chmm"))
    model = svh.DeviceModel(hmm)
    scores, best = svh.decode_file(model, ess("emit_50_3500_20.ess"), max_symbols=5 * 3500)  # 10 chunks
    g = load_golden("chmm2405_emit50")
    for rec in g["sequences"]:
        assert bit_equal(scores[rec["index"]], from_hex(rec["scores"]))
    one_s, one_b = model.viterbi(svh.read_emit_seq(ess("emit_50_3500_20.ess")))
    assert bit_equal(scores, one_s) and np.array_equal(best, one_b)


def test_decode_general_model_paths(tmp_path):
    """A model outside the chain kernel's shape: fused kernel + 16-bit backpointers, chunked."""
    hmm = random_hmm(300, out_degree=4, seed=3)
    seqs = random_seqs(hmm.emit_num, [1, 2, 50, 700, 64, 3], seed=3)
    p = tmp_path / "r.ess"
    p.write_text(ess_text([list(map(int, s)) for s in seqs]))
    model = svh.DeviceModel(hmm)
    assert model.info()["paths_kernel"] != _lib.SVH_KERNEL_CHAIN
    scores, best, paths = svh.decode_file(model, str(p), paths=True, max_seqs=2)
    for q, seq in enumerate(seqs):
        ref, ref_best, ref_path = oracle.decode(hmm, seq)
        assert bit_equal(scores[q], ref) and best[q] == ref_best and np.array_equal(paths[q], ref_path), q


def test_decode_errors_after_delivery(tmp_path):
    """A parse error mid-file: the chunks before it are delivered, then the call fails."""
    good = open(FASTA).read()
    p = tmp_path / "bad.fasta"
    p.write_text(good + ">bad\nACDZ\n")
    hmm = svh.read_HMM(chmm("100.chmm"))
    model = svh.DeviceModel(hmm)
    with pytest.raises(_lib.SvhError) as err:
        svh.decode_file(model, str(p), max_seqs=4)
    assert err.value.code == _lib.SVH_E_RANGE
