"""GPU parity of the _spec path vs the oracle's GraphBLAS_spec_impl restatement (bit-exact)."""
import numpy as np
import pytest

import spec_viterbi_amd as svh
from spec_viterbi_amd import _lib
from oracle import oracle
from tests.conftest import chmm, ess
from tests.helpers import (bit_equal, first_mismatch, from_hex, load_digests, load_golden, random_chain_hmm, random_hmm,
                           random_seqs)

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


def _neg_hmm(seed):
    """A random model with some negative scores (p > 1 in the reference's -log2 p terms): the
    on-chip level-2 kernel then keeps every term (no candidate pruning), still exact."""
    hmm = random_hmm(300, out_degree=3, dense_rows=(0, 7), seed=seed, zero_emis=0.05)
    rng = np.random.default_rng(seed)
    tp = hmm.trans_probs.copy()
    flip = rng.random(tp.size) < 0.2
    tp[flip & np.isfinite(tp)] *= -0.5
    hmm.trans_probs = tp
    em = hmm.emissions.copy()
    em[(rng.random(em.shape) < 0.1) & np.isfinite(em)] *= -1.0
    hmm.emissions = em
    return hmm


SPEC2_MODELS = {
    "chmm_gen": lambda: random_hmm(900, S=10, out_degree=3, seed=21),                # heavy rows of degree 5..10
    "dense_rows": lambda: random_hmm(257, out_degree=2, dense_rows=(5, 100), seed=22, zero_emis=0.05),
    "chain_ties": lambda: random_chain_hmm(700, S=8, seed=23, ties=True),            # exact ties everywhere
    "chain_inf": lambda: random_chain_hmm(1300, S=8, seed=24, inf_edges=0.2, zero_emis=0.1, feed_c=True),
    "chain_gap": lambda: random_chain_hmm(2600, S=4, seed=25, gap=1000, start=(0, 5)),  # R = 4 rows per thread
    "negative": lambda: _neg_hmm(26),                                                # pruning off
    "one_state": lambda: random_hmm(1, out_degree=1, seed=27),
}


@pytest.mark.parametrize("name", list(SPEC2_MODELS))
def test_spec2_on_chip_vs_oracle(name):
    """_spec level 2 evaluated on chip from the folded sparse matrices (spec2.hip, no dense
    products) against the oracle's product-based GraphBLAS_spec_impl restatement, bit-exact, on
    ragged sequences (chunks + a tail of 0 or 1 observations, lengths 1 and 2 included); the same
    batch on the dense-product path (SVH_MODEL_SPEC_DENSE) must agree bit for bit too."""
    hmm = SPEC2_MODELS[name]()
    S = int(hmm.emit_num)
    seqs = random_seqs(S, [1, 2, 3, 4, 5, 64, 257, 1000, 1501], seed=sum(map(ord, name)))
    model = svh.DeviceModel(hmm)
    model.spec_build(2)
    assert model.info()["spec_bytes"] == 0, "expected the on-chip level-2 kernel (no products)"
    got, best = model.viterbi(seqs, level=2)
    refs = oracle.viterbi_spec_batch(hmm, 2, seqs)  # the products built once
    for q, seq in enumerate(seqs):
        ref = refs[q]
        assert bit_equal(got[q], ref), (name, q, first_mismatch(got[q], ref))
        ref_best = int(np.argmin(ref)) if np.isfinite(ref).any() else -1
        assert best[q] == ref_best or not np.isfinite(ref).any(), (q, best[q], ref_best)
    if hmm.states_num <= 1400:
        dense = svh.DeviceModel(hmm, flags=_lib.SVH_MODEL_SPEC_DENSE)
        dense.spec_build(2)
        assert dense.info()["spec_bytes"] > 0
        got2, _ = dense.viterbi(seqs, level=2)
        for q in range(len(seqs)):
            assert bit_equal(got[q], got2[q]), (name, q, first_mismatch(got[q], got2[q]))


def test_spec2_large_model_takes_dense_path():
    """A model past the on-chip kernel's limits (n > 4096 states) keeps the dense products."""
    hmm = random_hmm(4200, S=3, out_degree=2, seed=31)
    seqs = random_seqs(3, [1, 40, 97], seed=31)
    model = svh.DeviceModel(hmm)
    model.spec_build(2)
    assert model.info()["spec_bytes"] > 0
    got, _ = model.viterbi(seqs, level=2)
    refs = oracle.viterbi_spec_batch(hmm, 2, seqs)
    for q in range(len(seqs)):
        assert bit_equal(got[q], refs[q]), (q, first_mismatch(got[q], refs[q]))
