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
    """BASELINE config 4: 2405.chmm x emit_50_3500_20.ess on the _spec level-2 path through the
    reference's interface (HIP_spec_impl; reference GraphBLAS_spec_impl.cpp:15-36, :68-80; the
    chunks' products evaluated on chip, nothing precomputed: the pipelined plan, pipe_l2.hip).
    All 50 sequences run in one batch and every row is compared bit-exact against the oracle's
    level-2 scores (computed offline by the oracle, which does form the products): rows 0..1
    against the committed vectors, all 50 against the SHA-256 digests of the oracle's float32 rows
    (tests/golden/make_golden.py spec2); every row also within the
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


def _near_tie_hmm(seed):
    """Heavy rows (degree ~600) whose candidate terms sit 0..17 ulps apart: every score is
    3 * (1 + k 2^-23) with k drawn from {0, 1, 2, 15, 16, 17}, so the sums c_m = fl(b_m + v_m) of a
    heavy row's terms crowd around its minimum within the on-chip kernel's 16-ulp pruning margin
    (spec2.hip theta_of).  Pins the pruning bound bit-exactly against the oracle where it is
    tightest."""
    hmm = random_hmm(600, S=6, out_degree=3, dense_rows=(0, 3, 9), seed=seed)
    rng = np.random.default_rng(seed)
    ks = np.array([0, 1, 2, 15, 16, 17], np.float64)

    def near(shape):
        return (3.0 * (1.0 + rng.choice(ks, size=shape) * 2.0 ** -23)).astype(np.float32)

    tp = hmm.trans_probs.copy()
    fin = np.isfinite(tp)
    tp[fin] = near(int(fin.sum()))
    hmm.trans_probs = tp
    em = hmm.emissions.copy()
    fin = np.isfinite(em)
    em[fin] = near(int(fin.sum()))
    hmm.emissions = em
    return hmm


SPEC2_MODELS = {
    "chmm_gen": lambda: random_hmm(900, S=10, out_degree=3, seed=21),                # heavy rows of degree 5..10
    "dense_rows": lambda: random_hmm(257, out_degree=2, dense_rows=(5, 100), seed=22, zero_emis=0.05),
    "chain_ties": lambda: random_chain_hmm(700, S=8, seed=23, ties=True),            # exact ties everywhere
    "chain_inf": lambda: random_chain_hmm(1300, S=8, seed=24, inf_edges=0.2, zero_emis=0.1, feed_c=True),
    "chain_gap": lambda: random_chain_hmm(2600, S=4, seed=25, gap=1000, start=(0, 5)),  # n = 2602: R = 3 rows per thread
    "chain_r4": lambda: random_chain_hmm(3600, S=4, seed=28, gap=1700, start=(0, 9)),  # n = 3602: R = 4 rows per thread
    "near_ties": lambda: _near_tie_hmm(29),                                          # candidates 0..17 ulps apart
    "negative": lambda: _neg_hmm(26),                                                # pruning off
    "one_state": lambda: random_hmm(1, out_degree=1, seed=27),
}


@pytest.mark.parametrize("pref", ["auto", "spec2"])
@pytest.mark.parametrize("name", list(SPEC2_MODELS))
def test_spec2_on_chip_vs_oracle(name, pref):
    """_spec level 2 evaluated on chip from the folded sparse matrices (no dense products) against
    the oracle's product-based GraphBLAS_spec_impl restatement, bit-exact, on ragged sequences
    (chunks + a tail of 0 or 1 observations, lengths 1 and 2 included): under AUTO (the MSV-shaped
    models run the chunks on the pipelined plan, pipe_l2.hip, with spec2_kernel re-running the rows
    it flags) and with spec2_kernel for every row (another kernel preference); the same batch on the
    dense-product path (SVH_MODEL_SPEC_DENSE) must agree bit for bit too."""
    hmm = SPEC2_MODELS[name]()
    S = int(hmm.emit_num)
    seqs = random_seqs(S, [1, 2, 3, 4, 5, 64, 257, 1000, 1501], seed=sum(map(ord, name)))
    model = svh.DeviceModel(hmm, kernel=_lib.SVH_KERNEL_AUTO if pref == "auto" else _lib.SVH_KERNEL_GENERIC)
    model.spec_build(2)
    assert model.info()["spec_bytes"] == 0, "expected the on-chip level-2 kernel (no products)"
    if pref == "spec2":
        assert model.batch(seqs[:1]).plan(2)["kernel"] == _lib.SVH_KERNEL_SPEC2
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


def test_spec2_pipe_headline_no_fallback():
    """BASELINE config 4 at level 2 on the pipelined latency plan (pipe_l2.hip, SVH_KERNEL_SPEC2_PIPE):
    every chunk of the 50 rows in one launch (5 workgroups per row), the one-observation tails on
    the step kernel; all 50 rows against the oracle's level-2 digests and no row handed to
    spec2_kernel (the speculated (F, m) terms and F's light terms never win on the reference data,
    so a fallback would hide a wrong pipelined row)."""
    import hashlib

    hmm = svh.read_HMM(chmm("2405.chmm"))
    seqs = svh.read_emit_seq(ess("emit_50_3500_20.ess"))
    model = svh.DeviceModel(hmm)
    model.spec_build(2)
    batch = model.batch(seqs)
    assert batch.plan(2)["kernel"] == _lib.SVH_KERNEL_SPEC2_PIPE
    for _ in range(2):  # a re-run of the same batch (scratch epochs, the flags of the last run)
        batch.run(2)
        got, best = batch.read()
        assert batch.fallbacks() == 0
        rows = load_digests()["2405.chmm x emit_50_3500_20.ess level 2"]
        bad = [q for q in range(50)
               if hashlib.sha256(np.ascontiguousarray(got[q], np.float32).tobytes()).hexdigest() != rows[q]["scores_sha256"]]
        assert not bad, bad
        assert np.array_equal(best, np.argmin(got, axis=1))


@pytest.mark.parametrize("n_states", [300, 1300])
def test_spec2_pipe_fallback_rows_match_oracle(n_states):
    """Models whose feeder row takes its light term (M -> N free): the pipelined level-2 pass flags
    those rows and spec2_kernel re-runs them from the first observation's state; every row still
    equals the oracle's level 2 bit for bit, and rows did fall back."""
    total = 0
    for seed in range(3):
        hmm = random_chain_hmm(n_states, S=8, seed=seed)
        rows, cols = hmm.trans_rows.astype(np.int64), hmm.trans_cols.astype(np.int64)
        probs = hmm.trans_probs.copy()
        probs[(cols == 0) & (rows != 0)] = np.float32(0.0)
        hmm.trans_probs = probs
        seqs = random_seqs(8, [700, 1, 2, 40, 333, 64], seed=seed)
        model = svh.DeviceModel(hmm)
        model.spec_build(2)
        batch = model.batch(seqs)
        assert batch.plan(2)["kernel"] == _lib.SVH_KERNEL_SPEC2_PIPE
        batch.run(2)
        got, _ = batch.read()
        total += batch.fallbacks()
        refs = oracle.viterbi_spec_batch(hmm, 2, seqs)
        for q in range(len(seqs)):
            assert bit_equal(got[q], refs[q]), (seed, q, first_mismatch(got[q], refs[q]))
    assert total > 0


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
