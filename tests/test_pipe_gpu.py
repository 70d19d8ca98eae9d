"""GPU parity of the pipelined chain kernels: the latency plan (pipe.hip, SVH_KERNEL_PIPE) and the
wide throughput plan (pipe_wide.hip, SVH_KERNEL_PIPE_WIDE: one position block per workgroup, one
sequence per wave); most tests run on both.

The kernel speculates that the feeder row N never takes its light-state term and checks that
exactly at every observation; a failing sequence is re-run by the serial chain kernel, so results
are bit-identical either way.  Because that fallback would also hide a wrong pipelined result,
every reference workload here asserts that no row fell back (`DeviceBatch.fallbacks() == 0`), and
random models whose N does take its light term assert that rows did fall back and still match.
"""
import numpy as np
import pytest

import spec_viterbi_amd as svh
from spec_viterbi_amd import _lib
from oracle import oracle
from tests.conftest import chmm, ess
from tests.helpers import (bit_equal, first_mismatch, from_hex, load_digests, load_golden, random_chain_hmm,
                           random_seqs)

pytestmark = pytest.mark.gpu
PIPES = [_lib.SVH_KERNEL_PIPE, _lib.SVH_KERNEL_PIPE_WIDE]
pipes = pytest.mark.parametrize("kern", PIPES, ids=["pipe", "pipew"])


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    assert _lib.device_count() > 0, "no HIP device visible (GPU tests must run on an MI355X)"


def run(hmm, seqs, kernel=_lib.SVH_KERNEL_PIPE, level=0):
    model = svh.DeviceModel(hmm, kernel=kernel)
    if level >= 2:
        model.spec_build(level)
    b = model.batch(seqs)
    b.run(level)
    s, best = b.read()
    plan = b.plan(level)
    return s, best, (b.fallbacks() if kernel in PIPES else 0), plan


def pipew_waves(info, nseq):
    """Sequences per workgroup of a wide launch (kernels.h pipew_waves_for)."""
    need = -(-nseq * info["pipew_blocks"] // info["cu_count"])
    return next((min(c, info["pipew_waves"]) for c in (1, 2, 4, 8, 12, 16) if c >= need), info["pipew_waves"])


def assert_same(s1, b1, s2, b2):
    for q in range(len(s1)):
        assert bit_equal(s1[q], s2[q]), (q, first_mismatch(s1[q], s2[q]))
    assert np.array_equal(b1, b2)


def oracle_check(hmm, seqs, scores, best):
    refs, _ = oracle.viterbi_batch(hmm, seqs)
    for q, seq in enumerate(seqs):
        ref = refs[q]
        assert bit_equal(scores[q], ref), (q, first_mismatch(scores[q], ref))
        ref_best = int(np.argmin(ref)) if np.isfinite(ref).any() else 0
        assert best[q] == ref_best, (q, best[q], ref_best)


@pipes
def test_pipe_headline_goldens_no_fallback(kern):
    """BASELINE config 3 (2405.chmm x emit_50_3500_20, all 50 sequences) on the pipelined kernel:
    the committed golden rows bit-exact, the whole batch equal to the serial chain kernel, and no
    row fell back."""
    g = load_golden("chmm2405_emit50")
    hmm = svh.read_HMM(chmm("2405.chmm"))
    seqs = svh.read_emit_seq(ess("emit_50_3500_20.ess"))
    s, b, fb, plan = run(hmm, seqs, kernel=kern)
    assert plan["kernel"] == kern
    assert fb == 0
    for rec in g["sequences"]:
        q = rec["index"]
        assert bit_equal(s[q], from_hex(rec["scores"])), first_mismatch(s[q], from_hex(rec["scores"]))
        assert b[q] == rec["best_state"]
    sc, bc, _, _ = run(hmm, seqs, kernel=_lib.SVH_KERNEL_CHAIN)
    assert_same(s, b, sc, bc)


def test_pipe_auto_selects_pipe_for_small_batches():
    hmm = svh.read_HMM(chmm("2405.chmm"))
    model = svh.DeviceModel(hmm)
    info = model.info()
    assert info["pipe_slots"] > 0 and info["pipe_groups"] > 1
    small = model.batch(random_seqs(20, [50] * 4, seed=1))
    assert small.plan()["kernel"] == _lib.SVH_KERNEL_DIAG  # the latency plan's range: the diagonal plan
    # the diagonal plan while its grid is resident at two workgroups per CU, the latency plan above
    assert info["diag_max_nseq"] == min(info["pipe_max_nseq"], 4 * (2 * info["cu_count"] // info["diag_ranges"])), info
    mid = model.batch(random_seqs(20, [8] * (info["diag_max_nseq"] + 1), seed=4))
    assert mid.plan()["kernel"] == _lib.SVH_KERNEL_PIPE
    forced = svh.DeviceModel(hmm, kernel=_lib.SVH_KERNEL_PIPE).batch(random_seqs(20, [50] * 4, seed=1))
    assert forced.plan()["kernel"] == _lib.SVH_KERNEL_PIPE
    wide = model.batch(random_seqs(20, [8] * (info["pipe_max_nseq"] + 1), seed=2))
    assert info["pipew_min_nseq"] == info["pipe_max_nseq"] + 1 and info["pipew_blocks"] == 5, info
    assert wide.plan()["kernel"] == _lib.SVH_KERNEL_PIPE_WIDE
    w = pipew_waves(info, info["pipe_max_nseq"] + 1)
    assert wide.plan()["threads"] == 64 * w and wide.plan()["slots"] == info["pipew_slots"]
    assert pipew_waves(info, 8000) == 16 and pipew_waves(info, 50) == 1
    # the chain kernel forced: its wide plan
    chain = svh.DeviceModel(hmm, kernel=_lib.SVH_KERNEL_CHAIN).batch(random_seqs(20, [8] * 300, seed=3))
    assert chain.plan()["kernel"] == _lib.SVH_KERNEL_CHAIN


@pytest.mark.parametrize("name,ess_name,nseq", [("2405.chmm", "emit_50_3500_20.ess", 100),
                                                 ("1001.chmm", "emit_3_3500_20.ess", 200),
                                                 ("100.chmm", "emit_3_3500_20.ess", 400)])
def test_pipe_auto_two_workgroups_per_cu(name, ess_name, nseq):
    """AUTO's latency plan past one workgroup per CU (runtime.cpp: pipe_max_nseq = 2 x CUs / G for
    scores-only batches): 100 sequences of 2405.chmm (G = 5, 500 workgroups), 200 of 1001.chmm
    (G = 2, 400) and 400 of 100.chmm (G = 1, 400) on 256 CUs.  Rows are the reference file's
    sequences and rotated copies of them (np.roll: the same symbol statistics, so the speculation
    holds as on the file); every row bit-exact against the oracle (the file rows of 2405 also
    against the committed digests), best states equal, no row fell back."""
    import hashlib

    hmm = svh.read_HMM(chmm(name))
    base = svh.read_emit_seq(ess(ess_name))
    seqs = [base[q % len(base)] if q < len(base) else np.roll(base[q % len(base)], 97 * (q // len(base)))
            for q in range(nseq)]
    if name == "100.chmm":  # 400 x 3500 x 101 states through the oracle: shorter rows keep it quick
        seqs = [s[: 1200 + 7 * q] for q, s in enumerate(seqs)]
    info = svh.DeviceModel(hmm).info()
    G = info["pipe_groups"]
    assert info["pipe_max_nseq"] == 2 * info["cu_count"] // G, info
    assert info["cu_count"] < nseq * G <= 2 * info["cu_count"], (nseq, G, info["cu_count"])
    # AUTO runs these batches on the diagonal plan (test_diag_gpu.py); the latency plan forced
    model = svh.DeviceModel(hmm, kernel=_lib.SVH_KERNEL_PIPE)
    batch = model.batch(seqs)
    assert batch.plan()["kernel"] == _lib.SVH_KERNEL_PIPE
    batch.run()
    s, b = batch.read()
    assert batch.fallbacks() == 0
    oracle_check(hmm, seqs, s, b)
    if name == "2405.chmm":
        rows = load_digests()[f"{name} x {ess_name}"]
        for q in range(len(base)):
            assert hashlib.sha256(np.ascontiguousarray(s[q]).tobytes()).hexdigest() == rows[q]["scores_sha256"], q
            assert b[q] == rows[q]["best_state"], q
    batch.close()
    model.close()


@pipes
@pytest.mark.parametrize("name", ["100.chmm", "500.chmm", "1001.chmm", "1509.chmm", "2050.chmm"])
def test_pipe_reference_models_vs_oracle(name, kern):
    hmm = svh.read_HMM(chmm(name))
    seqs = svh.read_emit_seq(ess("emit_3_3500_20.ess"))
    s, b, fb, _ = run(hmm, seqs, kernel=kern)
    assert fb == 0
    oracle_check(hmm, seqs[:1], s[:1], b[:1])
    sc, bc, _, _ = run(hmm, seqs, kernel=_lib.SVH_KERNEL_CHAIN)
    assert_same(s, b, sc, bc)


@pipes
def test_pipe_covid_ragged_no_fallback(kern):
    """BASELINE config 5's workload: 16 real protein sequences of 38..7096 observations (the wide
    plan: 16 ragged sequences in one workgroup per block)."""
    hmm = svh.read_HMM(chmm("2405.chmm"))
    seqs = svh.read_emit_seq(ess("covid-19.ess"))
    s, b, fb, _ = run(hmm, seqs, kernel=kern)
    assert fb == 0
    sc, bc, _, _ = run(hmm, seqs, kernel=_lib.SVH_KERNEL_CHAIN)
    assert_same(s, b, sc, bc)
    short = [q for q in range(len(seqs)) if len(seqs[q]) < 400]
    oracle_check(hmm, [seqs[q] for q in short], s[short], b[short])


@pipes
@pytest.mark.parametrize("L", [1, 2, 3, 31, 32, 33, 63, 64, 65, 95, 1023, 1024, 1025, 1057, 2049])
def test_pipe_sequence_lengths(L, kern):
    """Head (single observations up to a multiple of 32), body (groups of 8) and tail; symbol
    windows of 1024; three workgroups per sequence (latency plan, L = 700 light states) or
    three position blocks (wide plan, L = 1300)."""
    hmm = random_chain_hmm(700 if kern == _lib.SVH_KERNEL_PIPE else 1300, S=20, seed=L, n_from_m=False)
    seqs = random_seqs(20, [L, L + 5, max(1, L - 3)], seed=L)
    s, b, fb, plan = run(hmm, seqs, kernel=kern)
    assert (plan["pipe_groups"] if kern == _lib.SVH_KERNEL_PIPE else plan["pipew_blocks"]) >= 2 and fb == 0
    oracle_check(hmm, seqs, s, b)


@pipes
def test_pipe_long_sequence_many_ring_laps(kern):
    """A 60,000-observation sequence: the granule ring (256 slots) turns ~230 times, 59 symbol
    windows, five workgroups of one sequence in flight."""
    hmm = random_chain_hmm(2400, S=20, seed=3, n_from_m=False)
    seqs = random_seqs(20, [60000, 4000], seed=4)
    s, b, fb, plan = run(hmm, seqs, kernel=kern)
    assert fb == 0 and (plan["pipe_groups"] if kern == _lib.SVH_KERNEL_PIPE else plan["pipew_blocks"]) >= 4
    sc, bc, _, _ = run(hmm, seqs, kernel=_lib.SVH_KERNEL_CHAIN)
    assert_same(s, b, sc, bc)


@pipes
def test_pipe_fallback_rows_match_oracle(kern):
    """Models whose feeder row takes its light term (cheap M -> N): the speculation fails, those
    rows are re-run serially, and every score still matches the oracle.  The latency plan re-runs
    them inside the pass (pipe_rerun_row, by the row's combining workgroup: one workgroup per row at
    300 states, the last of two at 700), the wide plan on the serial chain kernel."""
    total_fb = 0
    for seed in range(8):
        hmm = random_chain_hmm(300 if seed < 6 else 700, S=8, seed=seed)
        # make M_j -> N nearly free so N's light term wins somewhere
        rows, cols = hmm.trans_rows.astype(np.int64), hmm.trans_cols.astype(np.int64)
        probs = hmm.trans_probs.copy()
        probs[(cols == 0) & (rows != 0)] = np.float32(0.0)
        hmm.trans_probs = probs
        seqs = random_seqs(8, [700, 1, 40, 333], seed=seed)
        s, b, fb, _ = run(hmm, seqs, kernel=kern)
        total_fb += fb
        oracle_check(hmm, seqs, s, b)
    assert total_fb > 0


@pytest.mark.parametrize("variant", [dict(self_n=False), dict(c_from_m=False), dict(self_c=False),
                                     dict(gap=37), dict(zero_emis=0.2), dict(ties=True), dict(inf_edges=0.1),
                                     dict(start=(0, 5, 301))])
@pipes
def test_pipe_chain_variants(variant, kern):
    hmm = random_chain_hmm(600, S=12, seed=11, **variant)
    seqs = random_seqs(12, [300, 64, 1, 97], seed=12)
    s, b, fb, _ = run(hmm, seqs, kernel=kern)
    oracle_check(hmm, seqs, s, b)


@pytest.mark.parametrize("waves", [1, 2, 4, 8, 12, 16])
def test_pipew_geometries(waves):
    """Wide plan with 1 .. 16 sequences per workgroup, the count the batch width selects (about
    one workgroup per CU): ragged batches, equal to the chain kernel, a sample against the oracle."""
    hmm = random_chain_hmm(1300, S=20, seed=23, n_from_m=False)
    info = svh.DeviceModel(hmm).info()
    nseq = waves * info["cu_count"] // info["pipew_blocks"]
    rng = np.random.default_rng(waves)
    lens = [500, 129, 2, 64, 1030] + list(rng.integers(1, 90, size=nseq - 5))
    seqs = random_seqs(20, lens, seed=24)
    s, b, fb, plan = run(hmm, seqs, kernel=_lib.SVH_KERNEL_PIPE_WIDE)
    assert pipew_waves(info, nseq) == waves and plan["threads"] == 64 * waves and fb == 0, plan
    sc, bc, _, _ = run(hmm, seqs, kernel=_lib.SVH_KERNEL_CHAIN)
    assert_same(s, b, sc, bc)
    sample = [0, 1, 2, 3, 4, nseq - 1]
    oracle_check(hmm, [seqs[q] for q in sample], s[sample], b[sample])


@pytest.mark.parametrize("geom", [(1, 4), (1, 8), (2, 4), (2, 8)])
def test_pipe_geometries(geom, monkeypatch):
    """The latency plan's other geometries (1 x 4, 1 x 8, 2 x 8: built only with -DSVH_PIPE_AB_ALL,
    AUTO plans 2 x 4) on a random chain model against the oracle."""
    if not _lib.pipe_variant_built(geom[0], geom[1], 0 if geom != (2, 4) else 4):
        pytest.skip(f"geometry {geom} is an A/B build's (-DSVH_PIPE_AB_ALL)")
    monkeypatch.setenv("SVH_PIPE_SM", str(geom[0]))
    monkeypatch.setenv("SVH_PIPE_WAVES", str(geom[1]))
    hmm = random_chain_hmm(1300, S=20, seed=21, n_from_m=False)
    seqs = random_seqs(20, [500, 129, 2], seed=22)
    s, b, fb, plan = run(hmm, seqs)
    assert (plan["slots"], plan["pipe_waves"]) == geom
    assert fb == 0
    oracle_check(hmm, seqs, s, b)


@pytest.mark.parametrize("tm", [0, 1, 2, 3, 4])
def test_pipe_table_modes(tm, monkeypatch):
    """Every step table mode of the latency plan (pipe_kernel.h TM: per-slot tables, pair tables by
    64-bit moves, indexed operands, packed feeder terms, both) on the headline rows against the
    goldens and on random chain models (ties, +inf edges, light starts, chain breaks, lengths around
    the group / window boundaries) against the oracle.  TM 1..3 are A/B builds' (-DSVH_PIPE_AB_ALL)."""
    if not _lib.pipe_variant_built(2, 4, tm):
        pytest.skip(f"table mode {tm} is an A/B build's (-DSVH_PIPE_AB_ALL)")
    monkeypatch.setenv("SVH_PIPE_TM", str(tm))
    import hashlib

    rows = load_digests()["2405.chmm x emit_50_3500_20.ess"]
    hmm = svh.read_HMM(chmm("2405.chmm"))
    seqs = svh.read_emit_seq(ess("emit_50_3500_20.ess"))
    s, b, fb, plan = run(hmm, seqs)
    assert plan["kernel"] == _lib.SVH_KERNEL_PIPE and fb == 0
    for q in range(len(seqs)):
        assert hashlib.sha256(np.ascontiguousarray(s[q]).tobytes()).hexdigest() == rows[q]["scores_sha256"], q
        assert b[q] == rows[q]["best_state"], q
    for k, kw in enumerate([dict(n_from_m=False), dict(ties=True), dict(inf_edges=0.1), dict(start=(0, 5, 301)),
                            dict(gap=37), dict(self_c=False)]):
        hmm = random_chain_hmm(1300, S=20, seed=40 + k, **kw)
        seqs = random_seqs(20, [1, 7, 8, 9, 33, 500, 1025, 2100], seed=50 + k)
        s, b, fb, plan = run(hmm, seqs)
        oracle_check(hmm, seqs, s, b)


@pipes
def test_pipe_spec_level2_tail(kern):
    """_spec level 2: the chunks run on the dense products, the tail on the pipelined kernel from
    device scores (begin > 0, v_in); bit-exact against the oracle's level-2 association."""
    hmm = svh.read_HMM(chmm("100.chmm"))
    seqs = svh.read_emit_seq(ess("emit_3_3500_20.ess"))
    seqs = [seqs[0][:301], seqs[1][:64], seqs[2][:2]]
    s, b, fb, plan = run(hmm, seqs, kernel=kern, level=2)
    for q, seq in enumerate(seqs):
        ref = oracle.viterbi_spec(hmm, 2, seq)
        assert bit_equal(s[q], ref), (q, first_mismatch(s[q], ref))


@pipes
def test_pipe_reruns_and_two_batches_share_nothing_stale(kern):
    """Launch epochs: re-running a batch, and a second batch of different lengths on the same
    model, never read another launch's boundary granules."""
    hmm = random_chain_hmm(900, S=20, seed=31, n_from_m=False)
    model = svh.DeviceModel(hmm, kernel=kern)
    a = model.batch(random_seqs(20, [900, 33], seed=32))
    bb = model.batch(random_seqs(20, [100, 2000, 5], seed=33))
    res = []
    for batch in (a, bb, a, bb, a):
        batch.run()
        res.append(batch.read())
        assert batch.fallbacks() == 0
    for i, j in ((0, 2), (2, 4), (1, 3)):
        assert_same(res[i][0], res[i][1], res[j][0], res[j][1])
    oracle_check(hmm, random_seqs(20, [900, 33], seed=32), res[0][0], res[0][1])


def test_pipew_wide_batch_equals_chain_and_oracle():
    """AUTO on a batch wider than the latency plan's range: the wide pipelined plan, every row equal
    to the chain kernel's wide plan, a sample bit-exact against the oracle (random symbols: rows
    whose speculation fails fall back, still exact)."""
    hmm = svh.read_HMM(chmm("2405.chmm"))
    model = svh.DeviceModel(hmm)
    rng = np.random.default_rng(17)
    lens = [1, 2, 31, 32, 33, 257, 1025] + list(rng.integers(1, 400, size=model.info()["pipew_min_nseq"] + 60))
    seqs = [rng.integers(0, hmm.emit_num, size=int(k)).astype(np.uint64) for k in lens]
    batch = model.batch(seqs)
    assert batch.plan()["kernel"] == _lib.SVH_KERNEL_PIPE_WIDE
    batch.run()
    s, b = batch.read()
    sc, bc, _, _ = run(hmm, seqs, kernel=_lib.SVH_KERNEL_CHAIN)
    assert_same(s, b, sc, bc)
    sample = [0, 1, 2, 3, 4, 5, 6, 100, len(seqs) - 1]
    oracle_check(hmm, [seqs[q] for q in sample], s[sample], b[sample])


@pytest.mark.parametrize("name", ["1301.chmm", "1901.chmm", "2365.chmm"])
def test_pipew_other_pfam_models_replicated(name):
    """Other Pfam models, the reference's emit_50 sequences replicated past the latency plan's
    range with synthetic copies (as bench.py --replicate): equal to the chain kernel."""
    hmm = svh.read_HMM(chmm(name))
    base = svh.read_emit_seq(ess("emit_50_3500_20.ess"))
    rng = np.random.default_rng(9)
    seqs = list(base) + [rng.integers(0, hmm.emit_num, size=len(x) // 4 + 1).astype(np.uint64) for x in base] * 3
    s, b, fb, plan = run(hmm, seqs, kernel=_lib.SVH_KERNEL_PIPE_WIDE)
    sc, bc, _, _ = run(hmm, seqs, kernel=_lib.SVH_KERNEL_CHAIN)
    assert_same(s, b, sc, bc)


@pipes
def test_pipe_spec3_tail_starting_at_256(kern):
    """Regression for the pipelined kernels' initial progress word: a `_spec`
    level-3 tail that starts at observation 256 (a multiple of 64 past the flow-control window)
    and runs two observations, on a plan with two workgroups (latency plan) or two position blocks
    (wide plan) per sequence.  Before the fix the producer's first flow-control wait and the
    consumer's first granule wait deadlocked (a bounded-wait give-up).  Checked bit-exact against
    the serial chain kernel at level 3 and within the reference's tolerance of the non-spec
    oracle."""
    hmm = svh.read_HMM(chmm("1001.chmm"))
    seq = svh.read_emit_seq(ess("emit_3_3500_20.ess"))[0][:258]
    model = svh.DeviceModel(hmm, kernel=kern)
    info = model.info()
    assert (info["pipe_groups"] if kern == _lib.SVH_KERNEL_PIPE else info["pipew_blocks"]) >= 2, info
    model.spec_build(3)
    batch = model.batch([seq])
    assert batch.plan(3)["kernel"] == kern
    batch.run(3)
    got, _ = batch.read()
    batch.close()
    model.close()
    chain = svh.DeviceModel(hmm, kernel=_lib.SVH_KERNEL_CHAIN)
    chain.spec_build(3)
    ref, _ = chain.viterbi([seq], level=3)
    chain.close()
    assert bit_equal(got[0], ref[0]), first_mismatch(got[0], ref[0])
    assert all(svh.almost_equal(a, b) for a, b in zip(got[0], oracle.viterbi(hmm, seq)))


@pipes
def test_pipe_10M_observations_multi_block_no_fault(kern):
    """A 10 M-observation sequence on a model of 2,400 light states (5 workgroups of the latency
    plan, 5 position blocks of the wide plan: 4 boundary exchanges per observation), so it meets
    millions of slow-path re-reads.  The wait budget is reset per 1,024-observation symbol window
    (a give-up sticks), so length alone never trips the fault word.  Bit-exact against the serial
    chain kernel, no fallback row, and the model and batch stay usable afterwards."""
    hmm = random_chain_hmm(2400, S=20, seed=41, n_from_m=False)
    seqs = random_seqs(20, [10_000_000], seed=42)
    model = svh.DeviceModel(hmm, kernel=kern)
    batch = model.batch(seqs)
    plan = batch.plan()
    assert plan["kernel"] == kern
    assert (plan["pipe_groups"] if kern == _lib.SVH_KERNEL_PIPE else plan["pipew_blocks"]) >= 4, plan
    batch.run()
    s, b = batch.read()
    assert batch.fallbacks() == 0
    batch.close()
    sc, bc, _, _ = run(hmm, seqs, kernel=_lib.SVH_KERNEL_CHAIN)
    assert_same(s, b, sc, bc)
    short = random_seqs(20, [3000], seed=43)
    s2, b2 = model.viterbi(short)
    oracle_check(hmm, short, s2, b2)
    model.close()


def test_fault_words_are_per_batch():
    """Two batches of one model on two streams; one is marked as if its bounded wait gave up
    (svh_batch_debug_fault).  Only that batch's read fails, once; the other batch's reads, before
    and after, succeed with correct scores, and the failed batch is judged on its own next run."""
    import torch

    hmm = random_chain_hmm(900, S=20, seed=51, n_from_m=False)
    model = svh.DeviceModel(hmm)
    seqs_a, seqs_b = random_seqs(20, [700, 33], seed=52), random_seqs(20, [100, 2000], seed=53)
    a, b = model.batch(seqs_a), model.batch(seqs_b)
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    a.run(0, sa.cuda_stream)
    b.run(0, sb.cuda_stream)
    b.debug_fault(sb.cuda_stream)
    ra = a.read(sa.cuda_stream)  # A must not see (or clear) B's fault
    oracle_check(hmm, seqs_a, *ra)
    with pytest.raises(_lib.SvhError):
        b.read(sb.cuda_stream)
    ra2 = a.read(sa.cuda_stream)
    oracle_check(hmm, seqs_a, *ra2)
    b.run(0, sb.cuda_stream)  # reported once: the next run of B is judged on its own
    rb = b.read(sb.cuda_stream)
    oracle_check(hmm, seqs_b, *rb)
    a.close()
    b.close()
    model.close()


def test_fallbacks_reset_by_time_parallel_run():
    """svh_batch_fallbacks reports the last run only: after a pipelined run() with fallback rows,
    a time-parallel pass (which never uses the pipelined kernel) reports 0."""
    for seed in range(6):  # the seeds of test_pipe_fallback_rows_match_oracle: some fall back
        hmm = random_chain_hmm(300, S=8, seed=seed)
        rows, cols = hmm.trans_rows.astype(np.int64), hmm.trans_cols.astype(np.int64)
        probs = hmm.trans_probs.copy()
        probs[(cols == 0) & (rows != 0)] = np.float32(0.0)
        hmm.trans_probs = probs
        model = svh.DeviceModel(hmm, kernel=_lib.SVH_KERNEL_PIPE)
        batch = model.batch(random_seqs(8, [700, 1, 40, 333], seed=seed))
        batch.run()
        batch.read()
        if batch.fallbacks() > 0:
            break
        batch.close()
        model.close()
    assert batch.fallbacks() > 0
    batch.run_time_parallel(seg_len=128, probe_len=16, rel_tol=-1.0)
    assert batch.fallbacks() == 0
    batch.close()
    model.close()


# ---- decoded paths on the pipelined plans (pipe_kernel.h / pipe_wide_kernel.h PATHS + pipe_paths.hip)
def decode_check(hmm, seqs, kernel=_lib.SVH_KERNEL_PIPE, expect_plan=True):
    """Scores, best states and paths of one decoded-path batch against the oracle's decode."""
    model = svh.DeviceModel(hmm, kernel=kernel)
    batch = model.batch(seqs, paths=True)
    plan = batch.plan()
    if expect_plan:
        assert plan["kernel"] == kernel, plan
    batch.run()
    s, b, pth = batch.read(want_paths=True)
    fb = batch.fallbacks()
    for q, seq in enumerate(seqs):
        ref, ref_best, ref_path = oracle.decode(hmm, seq)
        assert bit_equal(s[q], ref), (q, first_mismatch(s[q], ref))
        assert b[q] == ref_best, (q, b[q], ref_best)
        assert np.array_equal(pth[q], ref_path), (q, np.nonzero(pth[q] != ref_path)[0][:5], len(seq))
    batch.close()
    model.close()
    return fb


def test_pipe_paths_headline_digests():
    """BASELINE config 3 with decoded paths on the pipelined plan (AUTO): all 50 rows' scores and
    paths against the committed oracle digests, no fallback row."""
    import hashlib
    import json
    import os
    from tests.conftest import ROOT

    ref = json.load(open(os.path.join(ROOT, "tests", "golden", "score_digests.json")))
    hmm = svh.read_HMM(chmm("2405.chmm"))
    for ess_name in ("emit_50_3500_20.ess", "covid-19.ess"):
        seqs = svh.read_emit_seq(ess(ess_name))
        model = svh.DeviceModel(hmm)
        batch = model.batch(seqs, paths=True)
        assert batch.plan()["kernel"] == _lib.SVH_KERNEL_PIPE
        batch.run()
        s, b, pth = batch.read(want_paths=True)
        assert batch.fallbacks() == 0
        rows = ref[f"2405.chmm x {ess_name}"]
        for q in range(len(seqs)):
            assert hashlib.sha256(np.ascontiguousarray(s[q]).tobytes()).hexdigest() == rows[q]["scores_sha256"], q
            assert b[q] == rows[q]["best_state"]
            assert hashlib.sha256(np.asarray(pth[q], np.int32).tobytes()).hexdigest() == rows[q]["path_sha256"], q
        batch.close()
        model.close()


@pipes
@pytest.mark.parametrize("L", [1, 2, 3, 7, 8, 9, 16, 17, 31, 32, 33, 34, 63, 64, 65, 97, 1025, 2049])
def test_pipe_paths_sequence_lengths(L, kern):
    """Mask words (every 32 rows), checkpoints (every 16), ring folds (every 32 observations on the
    latency plan, every 8 on the wide plan) and the F checkpoints at every head / body / tail
    boundary; three workgroups (latency) or three blocks (wide) per sequence."""
    hmm = random_chain_hmm(700 if kern == _lib.SVH_KERNEL_PIPE else 1300, S=20, seed=L, n_from_m=False)
    decode_check(hmm, random_seqs(20, [L, L + 5, max(1, L - 3)], seed=L), kernel=kern)


@pytest.mark.parametrize("variant", [dict(), dict(self_n=False), dict(c_from_m=False), dict(self_c=False),
                                     dict(gap=37), dict(zero_emis=0.2), dict(ties=True), dict(inf_edges=0.1),
                                     dict(start=(0, 5, 301)), dict(n_from_m=False)])
@pipes
def test_pipe_paths_chain_variants(variant, kern):
    """MSV-shaped random models (ties, chain breaks, +inf edges, starts in light rows, no self
    loops): scores, best states and every path entry equal to the oracle's decode."""
    hmm = random_chain_hmm(600, S=12, seed=11, **variant)
    decode_check(hmm, random_seqs(12, [300, 64, 1, 97, 700], seed=12), kernel=kern)


@pipes
def test_pipe_paths_fallback_rows_match_oracle(kern):
    """Models whose feeder row takes its light term: those rows run on the chain kernel's path
    variant and its traceback, the others on the pipelined plan; every path equals the oracle's."""
    total_fb = 0
    for seed in range(6):
        hmm = random_chain_hmm(300 if kern == _lib.SVH_KERNEL_PIPE else 700, S=8, seed=seed)
        rows, cols = hmm.trans_rows.astype(np.int64), hmm.trans_cols.astype(np.int64)
        probs = hmm.trans_probs.copy()
        probs[(cols == 0) & (rows != 0)] = np.float32(0.0)
        hmm.trans_probs = probs
        total_fb += decode_check(hmm, random_seqs(8, [700, 1, 40, 333], seed=seed), kernel=kern)
    assert total_fb > 0


@pipes
@pytest.mark.parametrize("name", ["100.chmm", "1001.chmm", "2050.chmm"])
def test_pipe_paths_reference_models_vs_oracle(name, kern):
    hmm = svh.read_HMM(chmm(name))
    seqs = svh.read_emit_seq(ess("emit_3_3500_20.ess"))[:3]
    assert decode_check(hmm, seqs, kernel=kern) == 0


@pipes
def test_pipe_paths_covid_entries_through_match_states(kern):
    """covid-19 sequences whose best paths run N -> match states -> C (the j* recompute at the
    entry into C) on 2405.chmm, against the oracle's decode."""
    hmm = svh.read_HMM(chmm("2405.chmm"))
    seqs = svh.read_emit_seq(ess("covid-19.ess"))
    short = [s for s in seqs if len(s) < 1500][:4]
    assert decode_check(hmm, short, kernel=kern) == 0


@pytest.mark.parametrize("copies", [2, 8])
def test_pipew_paths_replicated_headline_digests(copies):
    """Wide path batches (AUTO past the latency plan's range: 100 and 400 sequences of
    2405.chmm x emit_50_3500_20, 2 and 8 sequences per workgroup): every row's scores, best state
    and path against the committed oracle digests, no fallback row."""
    import hashlib
    import json
    import os
    from tests.conftest import ROOT

    rows = json.load(open(os.path.join(ROOT, "tests", "golden", "score_digests.json")))[
        "2405.chmm x emit_50_3500_20.ess"]
    hmm = svh.read_HMM(chmm("2405.chmm"))
    seqs = svh.read_emit_seq(ess("emit_50_3500_20.ess")) * copies
    model = svh.DeviceModel(hmm)
    batch = model.batch(seqs, paths=True)
    plan = batch.plan()
    assert plan["kernel"] == _lib.SVH_KERNEL_PIPE_WIDE, plan
    batch.run()
    s, b, pth = batch.read(want_paths=True)
    assert batch.fallbacks() == 0
    for q in range(len(seqs)):
        r = rows[q % 50]
        assert hashlib.sha256(np.ascontiguousarray(s[q]).tobytes()).hexdigest() == r["scores_sha256"], q
        assert b[q] == r["best_state"], q
        assert hashlib.sha256(np.asarray(pth[q], np.int32).tobytes()).hexdigest() == r["path_sha256"], q
    batch.close()
    model.close()


def test_step_floor_measurement_and_untimed_batches():
    """svh_batch_step_floor_ms (the latency plan without its boundary exchange, bench.py's
    roofline.latency) returns a positive time below the real pass and leaves the batch's results,
    fault word and fallback flags untouched; a batch created with SVH_BATCH_NO_TIMING (timing=False)
    runs without its own events, reports fallbacks by waiting on the run's stream and refuses
    elapsed_ms()."""
    hmm = svh.read_HMM(chmm("2405.chmm"))
    seqs = svh.read_emit_seq(ess("emit_50_3500_20.ess"))
    model = svh.DeviceModel(hmm)
    batch = model.batch(seqs, timing=False)
    batch.run()
    s1, b1 = batch.read()
    floor = batch.step_floor_ms(5)
    assert floor > 0
    s2, b2 = batch.read()
    assert np.array_equal(s1.view(np.uint32), s2.view(np.uint32)) and np.array_equal(b1, b2)
    assert batch.fallbacks() == 0
    with pytest.raises(_lib.SvhError) as e:
        batch.elapsed_ms()
    assert e.value.code == _lib.SVH_E_STATE
    timed = model.batch(seqs)
    timed.run()
    assert floor < timed.elapsed_ms()
    g = load_golden("chmm2405_emit50")
    for rec in g["sequences"]:
        assert bit_equal(s1[rec["index"]], from_hex(rec["scores"]))
