"""GPU parity: the HIP path (through the C ABI) vs the oracle / committed goldens, bit-exact.

Scores must be bit-identical to GraphBLAS_impl's association (-0.0 == +0.0), best states and
decoded paths identical (lowest index on ties).
"""
import ctypes
import os

import numpy as np
import pytest

import spec_viterbi_amd as svh
from spec_viterbi_amd import _lib
from oracle import oracle
from tests.conftest import chmm, ess
from tests.helpers import (bit_equal, first_mismatch, from_hex, load_golden, random_chain_hmm, random_hmm,
                           random_seqs)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    assert _lib.device_count() > 0, "no HIP device visible (GPU tests must run on an MI355X)"


def check_against_oracle(hmm, seqs, kernel=_lib.SVH_KERNEL_AUTO, max_threads=0, paths=True):
    model = svh.DeviceModel(hmm, kernel=kernel, max_threads=max_threads)
    if paths:
        scores, best, pth = model.viterbi(seqs, paths=True)
    else:
        scores, best = model.viterbi(seqs)
    for q, seq in enumerate(seqs):
        if paths:
            ref, ref_best, ref_path = oracle.decode(hmm, seq)
        else:
            ref = oracle.viterbi(hmm, seq)
            ref_best = int(np.argmin(ref)) if np.isfinite(ref).any() else 0
        assert bit_equal(scores[q], ref), (q, first_mismatch(scores[q], ref), model.info())
        assert best[q] == ref_best, (q, best[q], ref_best)
        if paths:
            assert np.array_equal(pth[q], ref_path), (q, np.nonzero(pth[q] != ref_path)[0][:5])
    return model


@pytest.mark.parametrize("i", range(4))
def test_reference_fixtures(i):
    hmm = svh.read_HMM(chmm(f"test_chmms/{i}_test_chmm.chmm"))
    seqs = svh.read_emit_seq(ess(f"test_sequences/{i}_test_seq.ess"))
    check_against_oracle(hmm, seqs)
    check_against_oracle(hmm, seqs, kernel=_lib.SVH_KERNEL_GENERIC)


def test_cpp_interface_fixtures_through_python_mirror():
    impl = svh.HIP_impl()
    expected = load_golden("test_chmms")
    for i, case in enumerate(expected):
        hmm = svh.read_HMM(chmm(f"test_chmms/{i}_test_chmm.chmm"))
        seqs = svh.read_emit_seq(ess(f"test_sequences/{i}_test_seq.ess"))
        for rec in case["sequences"]:
            assert bit_equal(impl.run_Viterbi(hmm, seqs[rec["index"]]), from_hex(rec["scores"]))
            assert list(impl.decode_path(hmm, seqs[rec["index"]])) == rec["path"]


@pytest.mark.parametrize("name", ["chmm100_emit3", "chmm2405_emit50"])
def test_committed_goldens(name):
    g = load_golden(name)
    hmm = svh.read_HMM(chmm(g["chmm"].split("chmm_files/")[1]))
    seqs = svh.read_emit_seq(ess(g["ess"].split("ess_files/")[1]))
    idx = [r["index"] for r in g["sequences"]]
    model = svh.DeviceModel(hmm)
    scores, best, pth = model.viterbi([seqs[i] for i in idx], paths=True)
    for k, rec in enumerate(g["sequences"]):
        assert bit_equal(scores[k], from_hex(rec["scores"])), first_mismatch(scores[k], from_hex(rec["scores"]))
        assert best[k] == rec["best_state"]
        assert pth[k].tolist() == rec["path"]


def test_2405_emit50_full_batch_vs_oracle():
    """configs[2]: 2405.chmm x emit_50_3500_20 (all 50 sequences), non-spec path."""
    hmm = svh.read_HMM(chmm("2405.chmm"))
    seqs = svh.read_emit_seq(ess("emit_50_3500_20.ess"))
    model = svh.DeviceModel(hmm)
    batch = model.batch(seqs)
    plan = batch.plan()
    # AUTO takes the diagonal plan for this batch (13 groups of 4 sequences x 38 ranges)
    assert plan["kernel"] == _lib.SVH_KERNEL_DIAG and plan["diag_ranges"] == 38, plan
    batch.run()
    scores, best = batch.read()
    assert batch.fallbacks() == 0
    ref, _ = oracle.viterbi_batch(hmm, seqs, nthreads=16)
    for q in range(len(seqs)):
        assert bit_equal(scores[q], ref[q]), (q, first_mismatch(scores[q], ref[q]))
        assert best[q] == int(np.argmin(ref[q]))


@pytest.mark.parametrize("name", ["100.chmm", "200.chmm", "500.chmm", "1001.chmm", "1509.chmm", "2050.chmm",
                                  "2365.chmm"])
def test_pfam_models_emit3(name):
    hmm = svh.read_HMM(chmm(name))
    seqs = svh.read_emit_seq(ess("emit_3_3500_20.ess"))
    check_against_oracle(hmm, seqs[:2], paths=False)


def test_covid_ragged_batch():
    """configs[4] data: 16 sequences of lengths 38..7096 (> the 4096-symbol LDS ring)."""
    hmm = svh.read_HMM(chmm("2405.chmm"))
    seqs = svh.read_emit_seq(ess("covid-19.ess"))
    check_against_oracle(hmm, seqs, paths=False)


def test_paths_on_large_model():
    hmm = svh.read_HMM(chmm("900.chmm"))
    seqs = svh.read_emit_seq(ess("emit_3_3500_20.ess"))
    check_against_oracle(hmm, seqs[:1], paths=True)


@pytest.mark.parametrize("threads", [64, 128, 256, 512])
def test_workgroup_geometries(threads):
    hmm = svh.read_HMM(chmm("300.chmm"))
    seqs = svh.read_emit_seq(ess("emit_3_3500_20.ess"))
    check_against_oracle(hmm, [s[:700] for s in seqs], max_threads=threads)


@pytest.mark.parametrize("n,degree,dense,seed", [
    (900, 3, (), 1),          # chmm_gen.py shape: in-degree ~Poisson(3) -> R4/R8/R16 families
    (257, 2, (5,), 2),        # one dense row -> general heavy rows
    (300, 3, (0, 7, 299), 3),  # three dense rows -> R4+ families
    (64, 1, (), 4),
    (1, 1, (), 5),            # single state
])
def test_random_models(n, degree, dense, seed):
    hmm = random_hmm(n, out_degree=degree, dense_rows=dense, seed=seed, zero_emis=0.05)
    seqs = random_seqs(20, [1, 2, 3, 17, 500], seed=seed)
    check_against_oracle(hmm, seqs)
    check_against_oracle(hmm, seqs, kernel=_lib.SVH_KERNEL_GENERIC)


def test_high_indegree_falls_back_to_generic():
    hmm = random_hmm(200, out_degree=30, seed=9)  # in-degree ~30: no fused family fits
    model = check_against_oracle(hmm, random_seqs(20, [50, 300], seed=9))
    assert model.info()["kernel"] == _lib.SVH_KERNEL_GENERIC


def test_duplicate_transitions_first_wins():
    base = svh.read_HMM(chmm("test_chmms/3_test_chmm.chmm"))
    # duplicate (1 -> 2) with a different probability appended: GrB_FIRST keeps the original
    hmm = svh.HMM(states_num=base.states_num, emit_num=base.emit_num, trans_num=base.trans_num + 1,
                  trans_rows=np.append(base.trans_rows, 1), trans_cols=np.append(base.trans_cols, 2),
                  trans_probs=np.append(base.trans_probs, np.float32(0.01)), emissions=base.emissions,
                  start_probabilities_cols=np.append(base.start_probabilities_cols, 0),
                  start_probabilities=np.append(base.start_probabilities, np.float32(5.0)))
    seqs = svh.read_emit_seq(ess("test_sequences/3_test_seq.ess"))
    check_against_oracle(hmm, seqs)


def test_errors():
    hmm = svh.read_HMM(chmm("test_chmms/0_test_chmm.chmm"))
    model = svh.DeviceModel(hmm)
    with pytest.raises(_lib.SvhError) as e:
        model.viterbi([np.array([0, 4], np.uint64)])  # symbol 4 >= emit_num 4
    assert e.value.code == _lib.SVH_E_RANGE
    with pytest.raises(_lib.SvhError) as e:
        model.viterbi([np.array([], np.uint64)])
    assert e.value.code == _lib.SVH_E_INVALID
    with pytest.raises(_lib.SvhError) as e:
        model.viterbi([np.array([0, 1], np.uint64)], level=2)  # spec products not built
    assert e.value.code == _lib.SVH_E_STATE
    for kw in ({"kernel": _lib.SVH_KERNEL_SPEC2}, {"kernel": -1}, {"flags": 2}):  # not selectable / unknown bits
        with pytest.raises(_lib.SvhError) as e:
            svh.DeviceModel(hmm, **kw)
        assert e.value.code == _lib.SVH_E_INVALID


def test_spec2_plan_reported():
    """svh_batch_plan at level 2: an MSV-shaped model under AUTO runs the chunks on the pipelined
    latency plan (SVH_KERNEL_SPEC2_PIPE: 256 threads, 2 slots, nothing precomputed); with another
    kernel preference the on-chip chunk kernel (SVH_KERNEL_SPEC2) with its workgroup size, LDS and
    table bytes; level 0 of the same batch keeps the step kernel."""
    hmm = svh.read_HMM(chmm("100.chmm"))
    seqs = svh.read_emit_seq(ess("emit_3_3500_20.ess"))
    model = svh.DeviceModel(hmm)
    model.spec_build(2)
    batch = model.batch(seqs)
    p2, p0 = batch.plan(2), batch.plan(0)
    assert p2["kernel"] == _lib.SVH_KERNEL_SPEC2_PIPE and p2["threads"] == 256 and p2["slots"] == 2
    assert p2["spec_bytes"] == 0 and p2["spec_level"] == 2
    assert p0["kernel"] not in (_lib.SVH_KERNEL_SPEC2, _lib.SVH_KERNEL_SPEC2_PIPE)
    model = svh.DeviceModel(hmm, kernel=_lib.SVH_KERNEL_GENERIC)
    model.spec_build(2)
    p2 = model.batch(seqs).plan(2)
    assert p2["kernel"] == _lib.SVH_KERNEL_SPEC2 and p2["threads"] == 1024
    assert p2["lds_bytes"] > 0 and p2["spec_bytes"] > 0 and p2["spec_level"] == 2


def test_batch_api_device_resident_rerun():
    hmm = svh.read_HMM(chmm("2405.chmm"))
    seqs = svh.read_emit_seq(ess("emit_50_3500_20.ess"))[:4]
    model = svh.DeviceModel(hmm)
    batch = model.batch(seqs)
    batch.run()
    a, _ = batch.read()
    batch.run()
    b, _ = batch.read()
    assert bit_equal(a, b)
    assert batch.elapsed_ms() > 0
    ref, _ = oracle.viterbi_batch(hmm, seqs)
    assert bit_equal(a, ref)


def test_2405_chain_band_fused_kernels_bitwise():
    """The barrier-free chain kernel, the barrier chain kernel and the fused kernel agree bit for
    bit (and with the oracle)."""
    hmm = svh.read_HMM(chmm("2405.chmm"))
    seqs = [s[:1200] for s in svh.read_emit_seq(ess("emit_50_3500_20.ess"))[:6]]
    ref, _ = oracle.viterbi_batch(hmm, seqs)
    out = {}
    for k in (_lib.SVH_KERNEL_CHAIN, _lib.SVH_KERNEL_BAND, _lib.SVH_KERNEL_FUSED):
        model = svh.DeviceModel(hmm, kernel=k)
        assert model.info()["kernel"] == k
        out[k] = model.viterbi(seqs)
        assert bit_equal(out[k][0], ref), (k, first_mismatch(out[k][0][0], ref[0]))
    assert np.array_equal(out[_lib.SVH_KERNEL_CHAIN][1], out[_lib.SVH_KERNEL_FUSED][1])


@pytest.mark.parametrize("kernel", [_lib.SVH_KERNEL_CHAIN, _lib.SVH_KERNEL_BAND])
@pytest.mark.parametrize("threads", [64, 128, 256, 512])
def test_chain_geometries(kernel, threads):
    hmm = svh.read_HMM(chmm("1001.chmm") if threads >= 256 or kernel == _lib.SVH_KERNEL_BAND else chmm("200.chmm"))
    seqs = [s[:900] for s in svh.read_emit_seq(ess("emit_3_3500_20.ess"))]
    model = check_against_oracle(hmm, seqs, kernel=kernel, max_threads=threads, paths=False)
    assert model.info()["kernel"] == kernel


@pytest.mark.parametrize("L,kw,seed", [
    (1, {}, 1), (2, {}, 2), (63, {}, 3), (64, {}, 4), (65, {}, 5), (700, {}, 6), (2560, {}, 7),
    (4000, {}, 14),                                   # too long for the register kernel
    (300, {"feed_c": True}, 8),                       # light rows fed by both heavy rows
    (300, {"self_n": False, "self_c": False}, 9),     # no exceptions
    (300, {"c_from_m": False}, 10),                   # a heavy row without light sources
    (300, {"zero_emis": 0.2}, 11),                    # +inf emissions
    (300, {"start": (0, 5, 301)}, 12),                # start in light and heavy rows
    (300, {"gap": 150}, 13),                          # chain break (no predecessor term)
    (300, {"S": 40}, 15),                             # too many symbols for the register kernel
])
def test_chain_random_models(L, kw, seed):
    hmm = random_chain_hmm(L, seed=seed, **kw)
    S = kw.get("S", 20)
    seqs = random_seqs(S, [1, 2, 3, 4, 5, 77, 1000, 5000], seed=seed)
    model = svh.DeviceModel(hmm)
    info = model.info()
    if L >= 2:
        want = _lib.SVH_KERNEL_CHAIN if (L <= 2560 and S <= 32) else _lib.SVH_KERNEL_BAND
        assert info["kernel"] == want, info
    check_against_oracle(hmm, seqs, paths=False)
    if L >= 2:
        check_against_oracle(hmm, seqs, kernel=_lib.SVH_KERNEL_BAND, paths=False)
    check_against_oracle(hmm, seqs[:4], paths=True)


@pytest.mark.parametrize("L,kw,seed", [
    (1, {}, 1), (2, {}, 2), (63, {}, 3), (64, {}, 4), (65, {}, 5), (700, {}, 6), (2560, {}, 7),
    (300, {"self_n": False, "self_c": False}, 9),     # no heavy-heavy terms
    (300, {"c_from_m": False}, 10),                   # a heavy row without light sources
    (300, {"zero_emis": 0.2}, 11),                    # +inf emissions
    (300, {"start": (0, 5, 301)}, 12),                # start in light and heavy rows
    (300, {"gap": 150}, 13),                          # chain break (no predecessor term)
    (300, {"ties": True}, 17),                        # integer scores: ties everywhere
    (1000, {"ties": True, "zero_emis": 0.1}, 18),
    (300, {"inf_edges": 0.3}, 19),                    # terms of weight +inf
    (300, {"inf_edges": 0.3, "ties": True, "start": (0, 7)}, 20),
    (300, {"feed_c": True}, 8),                       # two heavy feeders: fused paths
])
def test_chain_decoded_paths(L, kw, seed):
    """Decoded paths from the chain kernel's compact records (light lane masks, heavy-row records,
    score checkpoints that the traceback recomputes j* from) and the speculative traceback: scores,
    best states and every path
    entry identical to the oracle's lexicographic (value, row) argmin, over lengths 1..5000."""
    hmm = random_chain_hmm(L, seed=seed, **kw)
    seqs = random_seqs(20, [1, 2, 3, 4, 5, 6, 7, 8, 9, 63, 64, 65, 77, 1000, 5000], seed=seed)
    # AUTO: the pipelined plan's path variant where the model has one (chain fallback), else the
    # chain or fused variant; then the chain variant forced
    model = check_against_oracle(hmm, seqs, paths=True)
    info = model.info()
    want = (_lib.SVH_KERNEL_FUSED if kw.get("feed_c") else
            _lib.SVH_KERNEL_PIPE if info["pipe_slots"] > 0 else _lib.SVH_KERNEL_CHAIN)
    if L >= 2:
        assert info["paths_kernel"] == want, info
    if L >= 2 and not kw.get("feed_c"):
        model = check_against_oracle(hmm, seqs, kernel=_lib.SVH_KERNEL_CHAIN, paths=True)
        assert model.info()["paths_kernel"] == _lib.SVH_KERNEL_CHAIN, model.info()


def test_chain_paths_covid_2405():
    """covid-19.ess (38..7096 observations, symbol refills) on 2405.chmm: chain decoded paths."""
    hmm = svh.read_HMM(chmm("2405.chmm"))
    seqs = svh.read_emit_seq(ess("covid-19.ess"))
    model = check_against_oracle(hmm, seqs, kernel=_lib.SVH_KERNEL_CHAIN, paths=True)
    assert model.info()["paths_kernel"] == _lib.SVH_KERNEL_CHAIN


@pytest.mark.parametrize("threads", [64, 128, 256, 512])
def test_chain_paths_geometries(threads):
    hmm = svh.read_HMM(chmm("300.chmm"))
    seqs = svh.read_emit_seq(ess("emit_3_3500_20.ess"))
    model = check_against_oracle(hmm, seqs, kernel=_lib.SVH_KERNEL_CHAIN, max_threads=threads, paths=True)
    assert model.info()["paths_kernel"] == _lib.SVH_KERNEL_CHAIN


def test_chain_paths_match_fused_paths():
    """The two decoded-path implementations agree on every reference .chmm (emit_3_3500_20)."""
    seqs = svh.read_emit_seq(ess("emit_3_3500_20.ess"))
    for name in sorted(os.listdir(os.path.dirname(chmm("2405.chmm")))):
        if not name.endswith(".chmm"):
            continue
        hmm = svh.read_HMM(chmm(name))
        try:
            a = svh.DeviceModel(hmm, kernel=_lib.SVH_KERNEL_CHAIN)
        except _lib.SvhError:  # not chain-shaped
            continue
        if a.info()["paths_kernel"] != _lib.SVH_KERNEL_CHAIN:
            continue
        b = svh.DeviceModel(hmm, kernel=_lib.SVH_KERNEL_FUSED)
        sa, ba, pa = a.viterbi(seqs, paths=True)
        sb, bb, pb = b.viterbi(seqs, paths=True)
        assert bit_equal(sa, sb) and np.array_equal(ba, bb), name
        for q in range(len(seqs)):
            assert np.array_equal(pa[q], pb[q]), (name, q)


def test_chain_covid_many_sequences_and_resume():
    """Ragged batch (38..7096) through the chain kernel; then the _spec level-2 tail, which resumes
    the chain kernel from device-resident scores (begin > 0)."""
    hmm = svh.read_HMM(chmm("300.chmm"))
    seqs = svh.read_emit_seq(ess("covid-19.ess"))
    model = check_against_oracle(hmm, seqs, paths=False)
    assert model.info()["kernel"] == _lib.SVH_KERNEL_CHAIN


def test_band_rejects_non_chain_models():
    hmm = random_hmm(300, out_degree=3, seed=3)
    for k in (_lib.SVH_KERNEL_BAND, _lib.SVH_KERNEL_CHAIN):
        with pytest.raises(_lib.SvhError) as e:
            svh.DeviceModel(hmm, kernel=k)
        assert e.value.code == _lib.SVH_E_UNSUPPORTED


def test_run_sharded_cli_covid_paths(tmp_path):
    """The sharded runner as one RCCL rank on this GPU: covid-19 x 2405, scores,
    best states and decoded paths gathered through run_sharded, checked against the oracle."""
    import subprocess
    import sys

    out = tmp_path / "res.npz"
    env = dict(os.environ, MASTER_PORT="29561")
    r = subprocess.run([sys.executable, "-m", "spec_viterbi_amd.run_sharded", "--model", chmm("2405.chmm"),
                        "--ess", ess("covid-19.ess"), "--paths", "--out", str(out)],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    res = np.load(out)
    hmm = svh.read_HMM(chmm("2405.chmm"))
    seqs = svh.read_emit_seq(ess("covid-19.ess"))
    offs = res["path_offsets"]
    for q in (0, 5, len(seqs) - 1):
        sc, best, path = oracle.decode(hmm, seqs[q])
        assert bit_equal(res["scores"][q], sc), first_mismatch(res["scores"][q], sc)
        assert int(res["best"][q]) == best
        assert np.array_equal(res["paths"][offs[q]:offs[q + 1]], path)


def test_wide_batch_streamed_plan_2405():
    """A batch with more sequences than CUs runs the wide chain plan (4 waves, streamed E, two
    workgroups per CU; forced: AUTO runs the wide pipelined plan there): bit-exact against the
    oracle, and against the same sequences run in batches narrow enough for the default plan; its
    lengths cover 1, the 8-observation group edges and the symbol-chunk refill."""
    hmm = svh.read_HMM(chmm("2405.chmm"))
    model = svh.DeviceModel(hmm, kernel=_lib.SVH_KERNEL_CHAIN)
    info = model.info()
    assert info["kernel"] == _lib.SVH_KERNEL_CHAIN and info["wide_threads"] == 256, info
    rng = np.random.default_rng(11)
    lens = [1, 2, 7, 8, 9, 15, 16, 17, 33] + list(rng.integers(1, 300, size=400))
    seqs = [rng.integers(0, hmm.emit_num, size=int(k)).astype(np.uint64) for k in lens]
    wide, wide_best = model.viterbi(seqs)
    narrow = np.concatenate([model.viterbi(seqs[k:k + 100])[0] for k in range(0, len(seqs), 100)])
    assert bit_equal(wide, narrow)
    for q in list(range(9)) + [100, 257, len(seqs) - 1]:
        ref = oracle.viterbi(hmm, seqs[q])
        assert bit_equal(wide[q], ref), (q, first_mismatch(wide[q], ref))
        assert wide_best[q] == int(np.argmin(ref)), q


def test_chain_long_sequence_no_fault():
    """A 10 M-observation sequence on 8 waves of the chain kernel (the most inter-wave waits per
    observation): the wait budget is reset per symbol chunk, so length alone never trips the fault
    word (round-1 budget was cumulative per sequence).  The chain kernel is forced and the batch's
    own plan asserted (AUTO would pick the one-wave pipelined plan, which never waits).  Scores
    bit-exact against the oracle."""
    hmm = svh.read_HMM(chmm("100.chmm"))
    rng = np.random.default_rng(7)
    seq = rng.integers(0, hmm.emit_num, size=10_000_000).astype(np.uint64)
    os.environ["SVH_CHAIN_WAVES"] = "8"
    try:
        model = svh.DeviceModel(hmm, kernel=_lib.SVH_KERNEL_CHAIN)
    finally:
        os.environ.pop("SVH_CHAIN_WAVES", None)
    batch = model.batch([seq])
    plan = batch.plan()
    assert plan["kernel"] == _lib.SVH_KERNEL_CHAIN and plan["threads"] == 512, plan
    batch.run()
    got, best = batch.read()
    batch.close()
    ref = oracle.viterbi(hmm, seq)
    assert bit_equal(got[0], ref), first_mismatch(got[0], ref)
    # and the model stays usable (no stale fault) on a second run
    got2, _ = model.viterbi([seq[:5000]])
    assert bit_equal(got2[0], oracle.viterbi(hmm, seq[:5000]))


def test_hip_impl_cache_follows_the_hmm_passed():
    """HIP_impl must always use the HMM passed in (reference semantics), even when a temporary
    HMM is freed and the next one reuses its address, or an HMM is modified in place."""
    impl = svh.HIP_impl()
    seq = svh.read_emit_seq(ess("emit_3_3500_20.ess"))[0][:300]
    for name in ("100.chmm", "200.chmm", "100.chmm", "300.chmm"):
        got = impl.run_Viterbi(svh.read_HMM(chmm(name)), seq)  # temporary HMM each time
        assert bit_equal(got, oracle.viterbi(svh.read_HMM(chmm(name)), seq)), name
    hmm = svh.read_HMM(chmm("100.chmm"))
    a = impl.run_Viterbi(hmm, seq)
    hmm.trans_probs = hmm.trans_probs + np.float32(0.5)  # in-place change of the same object
    b = impl.run_Viterbi(hmm, seq)
    assert bit_equal(b, oracle.viterbi(hmm, seq)) and not bit_equal(a, b)


@pytest.mark.parametrize("name", ["1301.chmm", "1509.chmm", "1901.chmm", "2365.chmm"])
def test_wide_plan_other_pfam_models(name):
    """The wide chain plan (the chain kernel's plan for batches of more sequences than CUs) on
    other eligible Pfam models: every sequence equal to narrow batches of the same sequences, a
    sample bit-exact against the oracle; svh_batch_plan names the plan each batch runs."""
    hmm = svh.read_HMM(chmm(name))
    model = svh.DeviceModel(hmm, kernel=_lib.SVH_KERNEL_CHAIN)
    info = model.info()
    if not info["wide_threads"]:
        pytest.skip(f"{name}: no wide plan ({info['threads']} threads narrow)")
    rng = np.random.default_rng(5)
    lens = [1, 8, 9, 17] + list(rng.integers(1, 200, size=info["cu_count"] + 40))
    seqs = [rng.integers(0, hmm.emit_num, size=int(k)).astype(np.uint64) for k in lens]
    batch = model.batch(seqs)
    plan = batch.plan()
    assert plan["threads"] == info["wide_threads"] and plan["slots"] == info["wide_slots"], plan
    batch.run()
    wide, wide_best = batch.read()
    small = model.batch(seqs[:100])  # narrow batches: the 8-wave chain plan
    sp = small.plan()
    assert sp["kernel"] == _lib.SVH_KERNEL_CHAIN and sp["threads"] == info["threads"], sp
    narrow = np.concatenate([model.viterbi(seqs[k:k + 100])[0] for k in range(0, len(seqs), 100)])
    assert bit_equal(wide, narrow)
    for q in [0, 1, 2, 3, 150, len(seqs) - 1]:
        ref = oracle.viterbi(hmm, seqs[q])
        assert bit_equal(wide[q], ref), (q, first_mismatch(wide[q], ref))
        assert wide_best[q] == int(np.argmin(ref)), q


def test_oneshot_batches_reused_across_calls():
    """svh_viterbi keeps its batches between calls (grow-only device buffers): shrinking and
    growing batches, a paths call, a rejected call and a level-1 call in between must each give
    the oracle's results."""
    hmm = svh.read_HMM(chmm("2405.chmm"))
    seqs = svh.read_emit_seq(ess("emit_50_3500_20.ess"))
    model = svh.DeviceModel(hmm)
    ref, _ = oracle.viterbi_batch(hmm, seqs, nthreads=16)
    short = [s[:700] for s in seqs[:3]]
    ref_short = [oracle.viterbi(hmm, s) for s in short]
    for batch, expect in ((seqs, ref), (short, ref_short), (seqs[:1], ref[:1]), (seqs, ref)):
        scores, best = model.viterbi(batch)
        for q in range(len(batch)):
            assert bit_equal(scores[q], expect[q]), (len(batch), q, first_mismatch(scores[q], expect[q]))
            assert best[q] == int(np.argmin(expect[q]))
    bad = [np.array([0, 1, 250], dtype=np.uint64)]
    with pytest.raises(_lib.SvhError):
        model.viterbi(bad)
    scores, best, pth = model.viterbi(short, paths=True)
    for q, s in enumerate(short):
        r, rb, rp = oracle.decode(hmm, s)
        assert bit_equal(scores[q], r) and best[q] == rb and np.array_equal(pth[q], rp), q
    scores, _ = model.viterbi(seqs[:7], level=1)
    for q in range(7):
        assert bit_equal(scores[q], ref[q]), q


def test_oneshot_symbol_forms_agree():
    """The three one-shot entry points -- separate uint64 arrays (svh_viterbi_seqs, what
    DeviceModel.viterbi and HIP_impl::run_Viterbi_batch call), packed uint64 (svh_viterbi) and
    packed uint8 (svh_viterbi_u8, the device format) -- give the oracle's scores, best states and
    paths, and the same error codes (out-of-range symbol, empty sequence, null pointers)."""
    import ctypes

    from spec_viterbi_amd.hmm import pack_sequences

    hmm = svh.read_HMM(chmm("2405.chmm"))
    seqs = [s[:L] for s, L in zip(svh.read_emit_seq(ess("covid-19.ess")), (1, 2, 31, 32, 33, 900, 1025, 64))]
    model = svh.DeviceModel(hmm)
    offs, sym64 = pack_sequences(seqs)
    got = {"seqs": model.viterbi(seqs, paths=True), "u64": model.viterbi_packed(offs, sym64, paths=True),
           "u8": model.viterbi_packed(offs, sym64.astype(np.uint8), paths=True)}
    for q, s in enumerate(seqs):
        r, rb, rp = oracle.decode(hmm, s)
        for name, (scores, best, pth) in got.items():
            assert bit_equal(scores[q], r) and best[q] == rb and np.array_equal(pth[q], rp), (name, q)
    # a list of non-uint64 arrays is converted, then runs the same path
    s32 = [np.asarray(s, np.int32) for s in seqs[:3]]
    assert all(bit_equal(a, b) for a, b in zip(model.viterbi(s32)[0], got["seqs"][0][:3]))
    bad = np.array([0, 1, 20], np.uint64)  # 20 >= emit_num
    for call in (lambda: model.viterbi([bad]),
                 lambda: model.viterbi_packed(np.array([0, 3], np.uint64), bad),
                 lambda: model.viterbi_packed(np.array([0, 3], np.uint64), bad.astype(np.uint8))):
        with pytest.raises(_lib.SvhError) as e:
            call()
        assert e.value.code == _lib.SVH_E_RANGE
    with pytest.raises(_lib.SvhError) as e:
        model.viterbi([seqs[0], np.array([], np.uint64)])
    assert e.value.code == _lib.SVH_E_INVALID
    lens = np.array([3], np.uint64)
    ptrs = np.zeros(1, np.uint64)
    rc = _lib.lib.svh_viterbi_seqs(model.handle, 0, 1, ptrs.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                                  lens.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), None, None, None)
    assert rc == _lib.SVH_E_INVALID  # a null sequence pointer
    # and the model still answers afterwards
    scores, best = model.viterbi(seqs)
    assert all(bit_equal(scores[q], got["seqs"][0][q]) for q in range(len(seqs)))


def test_results_into_pinned_buffers():
    """svh_batch_read / svh_viterbi_u8 into page-locked arrays (svh_host_alloc: the DMA engine
    writes the scores directly, no staging): the headline batch's rows equal the digests and the
    pageable path's results, repeated calls overwrite the same buffers, paths too."""
    import hashlib

    from spec_viterbi_amd.hmm import pack_sequences
    from tests.helpers import load_digests

    rows = load_digests()["2405.chmm x emit_50_3500_20.ess"]
    hmm = svh.read_HMM(chmm("2405.chmm"))
    seqs = svh.read_emit_seq(ess("emit_50_3500_20.ess"))
    model = svh.DeviceModel(hmm)
    offs, sym64 = pack_sequences(seqs)
    sym8 = sym64.astype(np.uint8)
    out = (svh.pinned_empty((len(seqs), model.n), np.float32), svh.pinned_empty(len(seqs), np.int64))
    for _ in range(2):
        out[0].fill(np.nan)
        out[1].fill(-7)
        s, b = model.viterbi_packed(offs, sym8, out=out)
        assert s is out[0] and b is out[1]
        for q in range(len(seqs)):
            assert hashlib.sha256(np.ascontiguousarray(s[q]).tobytes()).hexdigest() == rows[q]["scores_sha256"], q
            assert b[q] == rows[q]["best_state"], q
    sp, bp = model.viterbi_packed(offs, sym8)
    assert np.array_equal(sp.view(np.uint32), out[0].view(np.uint32)) and np.array_equal(bp, out[1])
    # a batch read with a pinned score buffer and a pinned path buffer
    short = [x[:300] for x in seqs[:4]]
    batch = model.batch(short, paths=True)
    batch.run()
    ref_s, ref_b, ref_p = batch.read(want_paths=True)
    ps = svh.pinned_empty((len(short), model.n), np.float32)
    pb = np.empty(len(short), np.int64)
    pp = svh.pinned_empty(sum(x.size for x in short), np.int32)
    _lib.check(_lib.lib.svh_batch_read(batch._h, None, ps.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                                       pb.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                                       pp.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))))
    assert np.array_equal(ps.view(np.uint32), ref_s.view(np.uint32)) and np.array_equal(pb, ref_b)
    assert np.array_equal(pp, np.concatenate(ref_p))
    with pytest.raises(ValueError):
        model.viterbi_packed(offs, sym8, out=(out[0][:3], out[1]))
