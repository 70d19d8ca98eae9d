"""GPU parity of the _spec path vs the oracle's GraphBLAS_spec_impl restatement (bit-exact)."""
import numpy as np
import pytest

import spec_viterbi_amd as svh
from spec_viterbi_amd import _lib
from oracle import oracle
from tests.conftest import chmm, ess
from tests.helpers import bit_equal, first_mismatch, from_hex, load_digests, load_golden, random_hmm, random_seqs

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("level", [0, 1, 2, 3])
@pytest.mark.parametrize("i", range(4))
def test_spec_fixtures(i, level):
    hmm = svh.read_HMM(chmm(f"test_chmms/{i}_test_chmm.chmm"))
    seqs = svh.read_emit_seq(ess(f"test_sequences/{i}_test_seq.ess"))
    impl = svh.HIP_spec_impl(level)
    impl.spec_with(hmm)
    for seq in seqs:
        got = impl.run_Viterbi_spec(seq)
        ref = oracle.viterbi_spec(hmm, max(level, 1), seq)
        assert bit_equal(got, ref), (first_mismatch(got, ref))


def test_spec_golden_100_level2():
    g = load_golden("chmm100_emit3")
    hmm = svh.read_HMM(chmm("100.chmm"))
    seqs = svh.read_emit_seq(ess("emit_3_3500_20.ess"))
    impl = svh.HIP_spec_impl(2)
    impl.spec_with(hmm)
    got = impl.run_Viterbi_spec_batch(seqs)
    for rec in g["sequences"]:
        assert bit_equal(got[rec["index"]], from_hex(rec["spec"]["2"]))


@pytest.mark.parametrize("level", [2, 3])
def test_spec_random_ragged(level):
    hmm = random_hmm(40, out_degree=3, dense_rows=(3,), seed=11)
    seqs = random_seqs(20, [1, 2, 3, 4, 5, 9, 64, 301], seed=11)
    model = svh.DeviceModel(hmm)
    model.spec_build(level)
    got, _ = model.viterbi(seqs, level=level)
    for q, seq in enumerate(seqs):
        ref = oracle.viterbi_spec(hmm, level, seq)
        assert bit_equal(got[q], ref), (q, first_mismatch(got[q], ref))


def test_spec_level2_500_model():
    hmm = svh.read_HMM(chmm("500.chmm"))
    seqs = svh.read_emit_seq(ess("emit_3_3500_20.ess"))
    model = svh.DeviceModel(hmm)
    model.spec_build(2)
    got, _ = model.viterbi(seqs, level=2)
    for q, seq in enumerate(seqs):
        ref = oracle.viterbi_spec(hmm, 2, seq)
        assert bit_equal(got[q], ref), (q, first_mismatch(got[q], ref))
        # and within the reference's tolerance of the non-spec answer
        assert all(svh.almost_equal(a, b) for a, b in zip(got[q], oracle.viterbi(hmm, seq)))


def test_spec_level2_2405_emit50_config4():
    """BASELINE config 4: 2405.chmm x emit_50_3500_20.ess on the _spec level-2 path (400 dense
    2407 x 2408 products, 9.3 GB of HBM; reference GraphBLAS_spec_impl.cpp:15-36, :68-80).
    All 50 sequences run in one batch and every row is compared bit-exact against the oracle's
    level-2 scores: rows 0..1 against the committed vectors, all 50 against the SHA-256 digests of
    the oracle's float32 rows (tests/golden/make_golden.py spec2); every row also within the
    reference's semantic-equality bound (HMM::almost_equal, |diff| <= 1) of the non-spec scores."""
    import hashlib

    g = load_golden("chmm2405_emit50")
    hmm = svh.read_HMM(chmm("2405.chmm"))
    seqs = svh.read_emit_seq(ess("emit_50_3500_20.ess"))
    impl = svh.HIP_spec_impl(2)
    impl.spec_with(hmm)
    got = impl.run_Viterbi_spec_batch(seqs)
    assert got.shape == (50, hmm.states_num)
    for rec in g["sequences"]:
        ref = from_hex(rec["spec"]["2"])
        assert bit_equal(got[rec["index"]], ref), (rec["index"], first_mismatch(got[rec["index"]], ref))
    rows = load_digests()["2405.chmm x emit_50_3500_20.ess level 2"]
    assert len(rows) == 50
    bad = [q for q in range(50)
           if hashlib.sha256(np.ascontiguousarray(got[q], np.float32).tobytes()).hexdigest() != rows[q]["scores_sha256"]]
    assert not bad, f"level-2 rows differing from the oracle digests: {bad}"
    nonspec = svh.DeviceModel(hmm).viterbi(seqs)[0]
    assert np.all(np.abs(got - nonspec) <= 1.0)
    assert not np.array_equal(got, nonspec)  # level 2 really took the product path
