"""GPU: the opt-in time-parallel pass against the oracle.

Not bit-exact by design (a converged segment's end is assembled from guess runs that start at
other magnitudes, so their fp32 roundings differ from the serial pass's), so the bar is the
reference's own tolerance, HMM::almost_equal (|d| <= 1.0, Viterbi_impl/HMM.h:43-49), plus a
relative 2e-5 (measured up to 1.4e-5: 0.32 at scores near 30000 after the 7096-step covid
sequence; basis runs start at 0, the serial pass at the start's magnitude); with rel_tol < 0 every segment is re-run and the result must be bit-exact (the
orchestration itself is then checked exactly)."""
import numpy as np
import pytest

import spec_viterbi_amd as svh
from spec_viterbi_amd import _lib
from oracle import oracle
from tests.conftest import chmm, ess
from tests.helpers import bit_equal, random_chain_hmm, random_hmm, random_seqs

pytestmark = pytest.mark.gpu


def close(a, b, rel=2e-5):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    fin = np.isfinite(b)
    d = np.abs(a[fin] - b[fin])
    return bool(np.array_equal(np.isfinite(a), fin) and np.all(d <= 1.0) and
                np.all(d <= rel * np.maximum(1.0, np.abs(b[fin]))))


def test_forced_fallback_is_bit_exact():
    hmm = svh.read_HMM(chmm("2405.chmm"))
    seqs = svh.read_emit_seq(ess("covid-19.ess"))
    model = svh.DeviceModel(hmm)
    batch = model.batch(seqs)
    fb = batch.run_time_parallel(seg_len=300, probe_len=40, rel_tol=-1.0)
    assert fb > 0
    scores, best = batch.read()
    one_s, one_b = model.viterbi(seqs)
    assert bit_equal(scores, one_s) and np.array_equal(best, one_b)


@pytest.mark.parametrize("seg,probe", [(1024, 256), (512, 128), (2000, 500)])
def test_covid_2405_within_tolerance(seg, probe):
    """The Pfam model converges through its heavy-row basis (N and C run from unit vectors; the
    match states' part is dominated within the probe), so no segment is re-run."""
    hmm = svh.read_HMM(chmm("2405.chmm"))
    seqs = svh.read_emit_seq(ess("covid-19.ess"))
    model = svh.DeviceModel(hmm)
    batch = model.batch(seqs)
    fb = batch.run_time_parallel(seg_len=seg, probe_len=probe)
    assert fb == 0
    scores, best = batch.read()
    for q, seq in enumerate(seqs):
        ref = oracle.viterbi(hmm, seq)
        assert close(scores[q], ref), (q, fb)
        assert best[q] == int(np.argmin(ref)), q


@pytest.mark.parametrize("L,seed", [(300, 1), (64, 2), (1000, 3)])
def test_random_chain_models_within_tolerance(L, seed):
    hmm = random_chain_hmm(L, seed=seed)
    seqs = random_seqs(20, [5000, 3000, 1, 77, 2500], seed=seed)
    model = svh.DeviceModel(hmm)
    batch = model.batch(seqs)
    batch.run_time_parallel(seg_len=700, probe_len=200)
    scores, best = batch.read()
    for q, seq in enumerate(seqs):
        ref = oracle.viterbi(hmm, seq)
        assert close(scores[q], ref), q


def test_converges_on_a_mixing_model():
    """Segments of an ergodic random model converge within the probe (rank convergence), so most
    are not re-run -- and the scores stay within tolerance of the oracle."""
    hmm = random_hmm(300, out_degree=4, seed=3)
    seqs = random_seqs(hmm.emit_num, [8000, 6000, 4000, 100], seed=5)
    model = svh.DeviceModel(hmm)
    batch = model.batch(seqs)
    fb = batch.run_time_parallel(seg_len=1024, probe_len=256)
    assert fb <= 3  # of 12 segments after the first ones
    scores, best = batch.read()
    for q, seq in enumerate(seqs):
        ref = oracle.viterbi(hmm, seq)
        assert close(scores[q], ref), q
        assert best[q] == int(np.argmin(ref)), q


def test_errors():
    hmm = svh.read_HMM(chmm("100.chmm"))
    model = svh.DeviceModel(hmm)
    seqs = svh.read_emit_seq(ess("emit_3_3500_20.ess"))
    with pytest.raises(_lib.SvhError) as e:
        model.batch(seqs, paths=True).run_time_parallel()
    assert e.value.code == _lib.SVH_E_UNSUPPORTED
    with pytest.raises(_lib.SvhError) as e:
        model.batch(seqs).run_time_parallel(seg_len=100, probe_len=100)
    assert e.value.code == _lib.SVH_E_INVALID


def test_sharded_runner_time_parallel():
    """run_sharded(time_parallel=...) on one gloo rank: the rank's batch takes the time-parallel
    pass (covid-19 on the Pfam model) and the gathered scores stay within tolerance."""
    import socket

    import torch.distributed as dist

    from spec_viterbi_amd.sharding import run_sharded

    hmm = svh.read_HMM(chmm("2405.chmm"))
    seqs = svh.read_emit_seq(ess("covid-19.ess"))
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        scores, best, paths, secs = run_sharded(hmm, seqs, time_parallel=(1024, 128))
    finally:
        dist.destroy_process_group()
    assert paths is None and secs > 0
    for q, seq in enumerate(seqs):
        ref = oracle.viterbi(hmm, seq)
        assert close(scores[q], ref), q
        assert best[q] == int(np.argmin(ref)), q
    with pytest.raises(ValueError):
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
        try:
            run_sharded(hmm, seqs[:2], paths=True, time_parallel=(1024, 128))
        finally:
            dist.destroy_process_group()


def test_time_parallel_rows_beyond_cu_count_run_the_wide_plan():
    """Short segments give more launch rows (segments x basis runs) than CUs, so the step
    launches of the time-parallel pass take the wide chain plan, with rows that start from
    v_in at observations > 0: forced re-runs must be bit-exact, converged runs within tolerance."""
    hmm = svh.read_HMM(chmm("2405.chmm"))
    seqs = svh.read_emit_seq(ess("covid-19.ess"))
    model = svh.DeviceModel(hmm)
    assert model.info()["wide_threads"], model.info()
    assert sum(len(s) for s in seqs) // 64 * 3 > model.info()["cu_count"]
    one_s, one_b = model.viterbi(seqs)
    batch = model.batch(seqs)
    fb = batch.run_time_parallel(seg_len=64, probe_len=32, rel_tol=-1.0)
    assert fb > model.info()["cu_count"] // 3
    scores, best = batch.read()
    assert bit_equal(scores, one_s) and np.array_equal(best, one_b)
    batch.run_time_parallel(seg_len=128, probe_len=64)
    scores, best = batch.read()
    for q in range(len(seqs)):
        assert close(scores[q], one_s[q]), q
