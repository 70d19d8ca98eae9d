"""CPU: pin the oracle to the reference's own fixtures, then to the committed goldens.

The reference's GraphBLAS backend cannot be built here (SuiteSparse:GraphBLAS absent), so the
oracle is pinned by the reference's golden fixtures (tests/test_helper.h:17-22, tolerance
HMM::almost_equal = 1.0) and reader unit tests (tests/test_chmm_reader.cpp,
tests/test_ess_reader.cpp).
"""
import numpy as np
import pytest

import spec_viterbi_amd as svh
from oracle import oracle
from tests.conftest import chmm, ess
from tests.helpers import bit_equal, from_hex, load_golden

m = svh.to_modified_prob
# reference tests/test_helper.h:17-22
EXPECTED = [
    [25.6574, 24.4874, m(0)],
    [m(0.04608), m(0.10752)],
    [m(0.00882), m(0.02646)],
    [m(0), m(0.00000282), m(0.0000181), m(0.00000605)],
]


def fixture(i):
    return (svh.read_HMM(chmm(f"test_chmms/{i}_test_chmm.chmm")),
            svh.read_emit_seq(ess(f"test_sequences/{i}_test_seq.ess"))[0])


@pytest.mark.parametrize("i", range(4))
def test_oracle_matches_reference_fixtures(i):
    hmm, seq = fixture(i)
    got = oracle.viterbi(hmm, seq)
    assert len(got) == len(EXPECTED[i])
    assert all(svh.almost_equal(a, b) for a, b in zip(got, EXPECTED[i])), (got, EXPECTED[i])


@pytest.mark.parametrize("i", range(4))
@pytest.mark.parametrize("level", [1, 2, 3])  # LEVELS_TO_TEST = 3, test_helper.h:23
def test_oracle_spec_matches_reference_fixtures(i, level):
    hmm, seq = fixture(i)
    got = oracle.viterbi_spec(hmm, level, seq)
    assert all(svh.almost_equal(a, b) for a, b in zip(got, EXPECTED[i]))


def test_reference_chmm_reader_values():
    # reference tests/test_chmm_reader.cpp:3-31
    h = svh.read_HMM(chmm("test_chmms/0_test_chmm.chmm"))
    assert h.states_num == 3 and h.non_zero_start_probs == 2 and h.emit_num == 4 and h.trans_num == 4
    assert list(h.start_probabilities_cols) == [0, 1]
    assert np.allclose(h.start_probabilities, [m(0.5), m(0.5)])
    assert np.allclose(h.emissions[:, 0], [m(0.2), m(0.3), m(0.3), m(0.2)])
    assert np.allclose(h.emissions[:, 1], [m(0.3), m(0.2), m(0.2), m(0.3)])
    assert np.allclose(h.emissions[:, 2], [m(0.3), m(0.2), m(0.2), m(0.3)])
    assert list(h.trans_rows) == [0, 0, 1, 1] and list(h.trans_cols) == [0, 1, 0, 1]
    assert np.allclose(h.trans_probs, [m(0.5), m(0.5), m(0.4), m(0.6)])


def test_reference_ess_reader_values():
    # reference tests/test_ess_reader.cpp:3-10
    s = svh.read_emit_seq(ess("test_sequences/0_test_seq.ess"))
    assert [list(map(int, x)) for x in s] == [[2, 2, 1, 0, 1, 3, 2, 0, 0], [3, 2, 1, 0]]


@pytest.mark.parametrize("name", ["test_chmms", "chmm100_emit3", "chmm2405_emit50"])
def test_oracle_reproduces_committed_goldens(name):
    g = load_golden(name)
    cases = g if isinstance(g, list) else [g]
    for c in cases:
        hmm = svh.read_HMM(chmm(c["chmm"].split("chmm_files/")[1]))
        seqs = svh.read_emit_seq(ess(c["ess"].split("ess_files/")[1]))
        for rec in c["sequences"]:
            seq = seqs[rec["index"]]
            if "path" in rec:
                scores, best, path = oracle.decode(hmm, seq)
                assert best == rec["best_state"]
                assert path.tolist() == rec["path"]
            else:
                scores = oracle.viterbi(hmm, seq)
            assert bit_equal(scores, from_hex(rec["scores"]))
            for L, bits in rec["spec"].items():
                assert bit_equal(oracle.viterbi_spec(hmm, int(L), seq), from_hex(bits))


def test_spec_level1_is_bit_identical_to_non_spec():
    hmm = svh.read_HMM(chmm("100.chmm"))
    for seq in svh.read_emit_seq(ess("emit_3_3500_20.ess")):
        assert bit_equal(oracle.viterbi(hmm, seq), oracle.viterbi_spec(hmm, 1, seq))


def test_spec_level2_within_reference_tolerance():
    # reference tests/test_semantic_equality.cpp:64-78 (almost_equal between spec levels)
    hmm = svh.read_HMM(chmm("100.chmm"))
    for seq in svh.read_emit_seq(ess("emit_3_3500_20.ess")):
        a, b = oracle.viterbi(hmm, seq), oracle.viterbi_spec(hmm, 2, seq)
        assert all(svh.almost_equal(x, y) for x, y in zip(a, b))


def test_path_is_consistent_with_scores():
    # the decoded path's own score equals the best final score
    hmm, seq = fixture(3)
    scores, best, path = oracle.decode(hmm, seq)
    start = dict(zip(map(int, hmm.start_probabilities_cols), hmm.start_probabilities))
    T = {(int(s), int(d)): p for s, d, p in zip(hmm.trans_rows, hmm.trans_cols, hmm.trans_probs)}
    acc = np.float32(hmm.emissions[seq[0], path[0]] + start[int(path[0])])
    for t in range(1, len(seq)):
        acc = np.float32(np.float32(hmm.emissions[seq[t], path[t]] + T[(int(path[t - 1]), int(path[t]))]) + acc)
    assert acc == scores[best]


def test_sweep2_digests_reproduce():
    """tests/golden/sweep2_digests.json (level 2 of the reference sweep's other files, checked by
    tools/bench_sweep.py on the GPU): the oracle reproduces the first row of a small model's cells."""
    import hashlib
    import json
    import os

    with open(os.path.join(os.path.dirname(__file__), "golden", "sweep2_digests.json")) as f:
        d = json.load(f)
    hmm = svh.read_HMM(chmm("100.chmm"))
    for name in ("emit_3_7000_20.ess", "covid-19.ess"):
        seq = svh.read_emit_seq(ess(name))[0]
        got = hashlib.sha256(np.ascontiguousarray(oracle.viterbi_spec(hmm, 2, seq), np.float32).tobytes()).hexdigest()
        assert got == d[f"100.chmm x {name} level 2"][0], name
