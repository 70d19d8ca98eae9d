"""GPU parity of the diagonal plan (diag.hip, SVH_KERNEL_DIAG): the latency plan's recurrence with
every lane on an anti-diagonal of the (position, observation) grid, so a position's chain input is
the lane's own previous score.  AUTO runs it for the scores-only batches the latency plan used to
take.

As for the pipelined plans, a row whose speculation fails is re-run exactly (here inside the same
launch), which would also hide a wrong result: reference workloads assert that no row fell back
(`DeviceBatch.fallbacks() == 0`), and models whose feeder row does take its light term assert that
rows fell back and still match the oracle.  The plan's own edges: the ring refill every 32 steps
(lengths around 32 / 64 / 96 / 128), the diagonals' wrap from the last position to position 0
(light rows a multiple of 64 and not), one, two and four sequences per workgroup (batches of
1, 2, 3, 5), dummy waves of a partial last group, ragged rows in one workgroup.
"""
import hashlib

import numpy as np
import pytest

import spec_viterbi_amd as svh
from spec_viterbi_amd import _lib
from oracle import oracle
from tests.conftest import chmm, ess
from tests.helpers import (bit_equal, first_mismatch, from_hex, load_digests, load_golden, random_chain_hmm,
                           random_seqs)

pytestmark = pytest.mark.gpu
DIAG = _lib.SVH_KERNEL_DIAG


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    assert _lib.device_count() > 0, "no HIP device visible (GPU tests must run on an MI355X)"


def run(hmm, seqs, kernel=DIAG):
    model = svh.DeviceModel(hmm, kernel=kernel)
    b = model.batch(seqs)
    b.run()
    s, best = b.read()
    plan = b.plan()
    fb = b.fallbacks() if kernel in (DIAG, _lib.SVH_KERNEL_PIPE, _lib.SVH_KERNEL_AUTO) else 0
    b.close()
    model.close()
    return s, best, fb, plan


def assert_same(s1, b1, s2, b2):
    for q in range(len(s1)):
        assert bit_equal(s1[q], s2[q]), (q, first_mismatch(s1[q], s2[q]))
    assert np.array_equal(b1, b2)


def oracle_check(hmm, seqs, scores, best):
    refs, _ = oracle.viterbi_batch(hmm, seqs)
    for q in range(len(seqs)):
        assert bit_equal(scores[q], refs[q]), (q, first_mismatch(scores[q], refs[q]))
        ref_best = int(np.argmin(refs[q])) if np.isfinite(refs[q]).any() else 0
        assert best[q] == ref_best, (q, best[q], ref_best)


def test_diag_headline_auto_goldens_digests_no_fallback():
    """BASELINE config 3 (2405.chmm x emit_50_3500_20) through AUTO: the diagonal plan, 38 ranges,
    four sequences per workgroup; the golden rows bit-exact, every row against the committed
    digests, no row fell back, twice on one batch."""
    g = load_golden("chmm2405_emit50")
    hmm = svh.read_HMM(chmm("2405.chmm"))
    seqs = svh.read_emit_seq(ess("emit_50_3500_20.ess"))
    model = svh.DeviceModel(hmm)
    info = model.info()
    assert info["diag_ranges"] == 38 and info["diag_max_nseq"] >= 50, info
    batch = model.batch(seqs)
    plan = batch.plan()
    assert plan["kernel"] == DIAG and plan["threads"] == 256 and plan["slots"] == 1, plan
    rows = load_digests()["2405.chmm x emit_50_3500_20.ess"]
    for _ in range(2):
        batch.run()
        s, b = batch.read()
        assert batch.fallbacks() == 0
        for rec in g["sequences"]:
            q = rec["index"]
            assert bit_equal(s[q], from_hex(rec["scores"])), first_mismatch(s[q], from_hex(rec["scores"]))
            assert b[q] == rec["best_state"]
        for q in range(len(seqs)):
            assert hashlib.sha256(np.ascontiguousarray(s[q]).tobytes()).hexdigest() == rows[q]["scores_sha256"], q
            assert b[q] == rows[q]["best_state"], q
    batch.close()
    model.close()


@pytest.mark.parametrize("nseq", [1, 2, 3, 5, 100])
def test_diag_workgroup_widths_vs_pipe(nseq):
    """1, 2 and 4 sequences per workgroup and a partial last group (3: two groups of two, one wave
    idle; 5: two groups of four, three waves idle); 100 rows of 2405.chmm (the file's 50 and rotated
    copies: 25 groups x 38 ranges, ~4 workgroups per CU), equal to the pipelined latency plan and the
    chain kernel, no fallback."""
    hmm = svh.read_HMM(chmm("2405.chmm"))
    base = svh.read_emit_seq(ess("emit_50_3500_20.ess"))
    seqs = [base[q] if q < len(base) else np.roll(base[q % len(base)], 97) for q in range(nseq)]
    s, b, fb, plan = run(hmm, seqs)
    assert plan["kernel"] == DIAG and plan["threads"] == 64 * (4 if nseq >= 4 else 2 if nseq >= 2 else 1), plan
    assert fb == 0
    sc, bc, _, _ = run(hmm, seqs, kernel=_lib.SVH_KERNEL_CHAIN)
    assert_same(s, b, sc, bc)
    if nseq <= 5:
        sp, bp, _, _ = run(hmm, seqs, kernel=_lib.SVH_KERNEL_PIPE)
        assert_same(s, b, sp, bp)


@pytest.mark.parametrize("name", ["100.chmm", "500.chmm", "1001.chmm", "1509.chmm", "2050.chmm", "2405.chmm"])
def test_diag_reference_models(name):
    """Reference models under AUTO with emit_3 (3 sequences: two groups, two waves each): equal to
    the chain kernel, one row against the oracle, no fallback."""
    hmm = svh.read_HMM(chmm(name))
    seqs = svh.read_emit_seq(ess("emit_3_3500_20.ess"))
    s, b, fb, plan = run(hmm, seqs, kernel=_lib.SVH_KERNEL_AUTO)
    assert plan["kernel"] == DIAG and fb == 0, plan
    oracle_check(hmm, seqs[:1], s[:1], b[:1])
    sc, bc, _, _ = run(hmm, seqs, kernel=_lib.SVH_KERNEL_CHAIN)
    assert_same(s, b, sc, bc)


def test_diag_covid_ragged():
    """BASELINE config 5's workload: 16 real protein sequences of 38..7096 observations -- ragged
    rows in one workgroup (waves whose row has ended keep refilling the shared ring)."""
    hmm = svh.read_HMM(chmm("2405.chmm"))
    seqs = svh.read_emit_seq(ess("covid-19.ess"))
    s, b, fb, _ = run(hmm, seqs)
    assert fb == 0
    sc, bc, _, _ = run(hmm, seqs, kernel=_lib.SVH_KERNEL_CHAIN)
    assert_same(s, b, sc, bc)
    short = [q for q in range(len(seqs)) if len(seqs[q]) < 400]
    oracle_check(hmm, [seqs[q] for q in short], s[short], b[short])


@pytest.mark.parametrize("L", [1, 2, 3, 31, 32, 33, 34, 63, 64, 65, 95, 96, 97, 127, 128, 129, 1025, 2049])
def test_diag_sequence_lengths(L):
    """Lengths around the block of 32 steps (the ring refill and the stream double buffer), the
    ring of 128 columns, and longer; 700 light states (11 ranges, 60 dummy positions)."""
    hmm = random_chain_hmm(700, S=20, seed=L, n_from_m=False)
    seqs = random_seqs(20, [L, L + 5, max(1, L - 3), L + 33, 2 * L + 1], seed=L)
    s, b, fb, _ = run(hmm, seqs)
    assert fb == 0
    oracle_check(hmm, seqs, s, b)


@pytest.mark.parametrize("L", [62, 64, 126, 128, 129, 190, 1])
def test_diag_wrap_light_rows(L):
    """The diagonals' wrap: light rows a multiple of 64 (no dummy position: the lane goes from the
    last light row straight to position 0) and not; one range (L < 64) and several; sequences
    longer than the rows so every lane wraps many times."""
    hmm = random_chain_hmm(L, S=6, seed=100 + L, n_from_m=False)
    seqs = random_seqs(6, [3 * (L + 2) + 5, 700, 64], seed=L)
    s, b, fb, _ = run(hmm, seqs)
    assert fb == 0
    oracle_check(hmm, seqs, s, b)


def test_diag_long_sequence():
    """A 60,000-observation sequence beside a 4,000 one (1,875 blocks, the ring turns ~470 times)."""
    hmm = random_chain_hmm(2400, S=20, seed=3, n_from_m=False)
    seqs = random_seqs(20, [60000, 4000], seed=4)
    s, b, fb, _ = run(hmm, seqs)
    assert fb == 0
    sc, bc, _, _ = run(hmm, seqs, kernel=_lib.SVH_KERNEL_CHAIN)
    assert_same(s, b, sc, bc)


def test_diag_fallback_rows_match_oracle():
    """Models whose feeder row takes its light term (M -> N free): the speculation fails, the
    combining wave's workgroup re-runs those rows in the same launch, every score matches the
    oracle; rows of 1, 2 and 4 sequences per workgroup."""
    total_fb = 0
    for seed in range(8):
        hmm = random_chain_hmm(300 if seed < 6 else 700, S=8, seed=seed)
        rows, cols = hmm.trans_rows.astype(np.int64), hmm.trans_cols.astype(np.int64)
        probs = hmm.trans_probs.copy()
        probs[(cols == 0) & (rows != 0)] = np.float32(0.0)
        hmm.trans_probs = probs
        lens = [[700], [700, 1], [700, 1, 40, 333, 64]][seed % 3]
        seqs = random_seqs(8, lens, seed=seed)
        s, b, fb, _ = run(hmm, seqs)
        total_fb += fb
        oracle_check(hmm, seqs, s, b)
    assert total_fb > 0


@pytest.mark.parametrize("variant", [dict(self_n=False), dict(c_from_m=False), dict(self_c=False),
                                     dict(gap=37), dict(zero_emis=0.2), dict(ties=True), dict(inf_edges=0.1),
                                     dict(start=(0, 5, 301)), dict(sx=True)])
def test_diag_chain_variants(variant):
    """Chain-shaped edge cases: no self loops, no sink term, chain breaks, +inf emissions and edges,
    exact ties, starts in light rows, S fed by N (the X_SF term)."""
    hmm = random_chain_hmm(600, S=12, seed=11, **variant)
    if variant.get("sx"):  # N -> C: the sink takes a term from the feeder row (PipeModel.sx)
        hmm.trans_rows = np.append(hmm.trans_rows, np.uint64(0))
        hmm.trans_cols = np.append(hmm.trans_cols, np.uint64(hmm.states_num - 1))
        hmm.trans_probs = np.append(hmm.trans_probs, np.float32(3.5))
        hmm.trans_num += 1
    seqs = random_seqs(12, [300, 64, 1, 97, 33], seed=12)
    s, b, fb, plan = run(hmm, seqs)
    assert plan["kernel"] == DIAG
    oracle_check(hmm, seqs, s, b)


@pytest.mark.parametrize("S", [1, 2, 32])
def test_diag_alphabets(S):
    """One symbol (a single ring plane), two, and the 32-symbol maximum (ring 48 KB)."""
    hmm = random_chain_hmm(400, S=S, seed=40 + S, n_from_m=False)
    seqs = random_seqs(S, [250, 33, 96], seed=S)
    s, b, fb, _ = run(hmm, seqs)
    assert fb == 0
    oracle_check(hmm, seqs, s, b)


def test_diag_two_batches_two_streams():
    """Two headline batches in flight on two streams at once (each its own scratch and partials;
    988 workgroups against 256 CUs, so the second launch waits for CUs the first holds)."""
    import torch

    hmm = svh.read_HMM(chmm("2405.chmm"))
    seqs = svh.read_emit_seq(ess("emit_50_3500_20.ess"))
    rows = load_digests()["2405.chmm x emit_50_3500_20.ess"]
    model = svh.DeviceModel(hmm)
    a, b = model.batch(seqs), model.batch(seqs[::-1])
    assert a.plan()["kernel"] == DIAG
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    for _ in range(3):
        a.run(0, sa.cuda_stream)
        b.run(0, sb.cuda_stream)
        r1, k1 = a.read(sa.cuda_stream)
        r2, k2 = b.read(sb.cuda_stream)
        assert a.fallbacks() == 0 and b.fallbacks() == 0
        assert_same(r1, k1, r2[::-1], k2[::-1])
        for q in range(len(seqs)):
            assert hashlib.sha256(np.ascontiguousarray(r1[q]).tobytes()).hexdigest() == rows[q]["scores_sha256"], q
    a.close()
    b.close()
    model.close()


@pytest.mark.parametrize("kern", [DIAG, _lib.SVH_KERNEL_AUTO])
def test_diag_spec_tail_resumes_from_device_scores(kern):
    """_spec level 2: the chunks run on the dense products (DIAG) or on the latency plan's level-2
    kernel (AUTO); the tail -- rows resumed at begin > 0 from the chunks' device scores (v_in) -- on
    the diagonal plan.  Tails of 0 and 1 observations, a length-1 row (no chunk); bit-exact against
    the oracle's level-2 association.  (The level-2 rocprof trace, profiles/r06_m2, shows the tail's
    diag_viterbi_kernel launch.)"""
    hmm = svh.read_HMM(chmm("100.chmm"))
    base = svh.read_emit_seq(ess("emit_3_3500_20.ess"))
    seqs = [base[0][:301], base[1][:64], base[2][:2], base[0][:1], base[1][:1000]]
    model = svh.DeviceModel(hmm, kernel=kern)
    model.spec_build(2)
    batch = model.batch(seqs)
    batch.run(2)
    s, _ = batch.read()
    batch.close()
    model.close()
    for q, seq in enumerate(seqs):
        ref = oracle.viterbi_spec(hmm, 2, seq)
        assert bit_equal(s[q], ref), (q, first_mismatch(s[q], ref))


def test_diag_spec3_tail_equals_chain():
    """_spec level 3 (tails of 0, 1 and 2 observations, one starting at 256) on the diagonal plan
    against the serial chain kernel at level 3, bit-exact."""
    hmm = svh.read_HMM(chmm("1001.chmm"))
    base = svh.read_emit_seq(ess("emit_3_3500_20.ess"))
    seqs = [base[0][:258], base[1][:259], base[2][:260], base[0][:3]]
    out = []
    for kern in (DIAG, _lib.SVH_KERNEL_CHAIN):
        model = svh.DeviceModel(hmm, kernel=kern)
        model.spec_build(3)
        out.append(model.viterbi(seqs, level=3))
        model.close()
    assert_same(out[0][0], out[0][1], out[1][0], out[1][1])
