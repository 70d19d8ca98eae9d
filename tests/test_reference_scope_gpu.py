"""GPU parity over the reference's own model scope, on the product kernels AUTO selects.

The reference's semantic-equality test runs every `.chmm` against every sequence of
`emit_3_3500_20.ess`, non-spec and `_spec` levels 1 and 2 (tests/test_semantic_equality.cpp:19-98),
and its harness benchmarks every `.chmm` (benchmark/bench_Viterbi.h:37-48).  Here the same 24 x 3
rows run through AUTO (the pipelined latency plan: G = 1..5 workgroups per sequence across the
models) and are compared bit-exact with the oracle's committed digests
(tests/golden/scope_digests.json, `make_golden.py scope`): scores, best states, the decoded path of
every row, and the level-2 scores (the reference compares levels only within +-1.0; the oracle's
level-2 association is exact).  Also: two headline batches launched at once on two streams, whose
grids together exceed the CUs.
"""
import glob
import hashlib
import json
import os

import numpy as np
import pytest

import spec_viterbi_amd as svh
from spec_viterbi_amd import _lib
from tests.conftest import DATA, chmm, ess
from tests.helpers import GOLDEN, load_digests

pytestmark = pytest.mark.gpu

MODELS = sorted((os.path.basename(f) for f in glob.glob(os.path.join(DATA, "chmm_files", "*.chmm"))),
                key=lambda f: int(f.split(".")[0]))


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    assert _lib.device_count() > 0, "no HIP device visible (GPU tests must run on an MI355X)"


@pytest.fixture(scope="module")
def scope():
    with open(os.path.join(GOLDEN, "scope_digests.json")) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def emit3():
    return svh.read_emit_seq(ess("emit_3_3500_20.ess"))


def sha(a, dt):
    return hashlib.sha256(np.ascontiguousarray(a, dt).tobytes()).hexdigest()


def expected_groups(n):
    """Workgroups per sequence of the latency plan for an MSV model of n states: light positions
    in blocks of 128 (2 slots x 64 lanes), 4 blocks (waves) per workgroup."""
    blocks = -(-(n - 2) // 128)
    return -(-blocks // 4)


def test_scope_covers_every_model_and_geometry(scope):
    assert len(MODELS) == 24 and sorted(scope["models"]) == sorted(MODELS)
    groups = {expected_groups(svh.read_HMM(chmm(m)).states_num) for m in MODELS}
    assert groups == {1, 2, 3, 4, 5}, groups


@pytest.mark.parametrize("name", MODELS)
def test_scope_scores_and_paths(name, scope, emit3):
    """Every emit_3 row of this model: scores and best states on one AUTO batch (the diagonal plan,
    its ranges named) and on the latency plan forced (G named), then every row's decoded path (AUTO:
    the latency plan's path variant); no row may fall back to the serial kernel."""
    hmm = svh.read_HMM(chmm(name))
    ref = scope["models"][name]
    forced = svh.DeviceModel(hmm, kernel=_lib.SVH_KERNEL_PIPE)
    model = svh.DeviceModel(hmm)
    for m, kern in ((model, _lib.SVH_KERNEL_DIAG), (forced, _lib.SVH_KERNEL_PIPE)):
        batch = m.batch(emit3)
        plan = batch.plan()
        assert plan["kernel"] == kern, plan
        if kern == _lib.SVH_KERNEL_PIPE:
            assert plan["pipe_groups"] == expected_groups(hmm.states_num), plan
        else:
            assert plan["diag_ranges"] == -(-(hmm.states_num - 2) // 64), plan
        batch.run()
        scores, best = batch.read()
        assert batch.fallbacks() == 0
        for q in range(len(emit3)):
            assert sha(scores[q], np.float32) == ref[q]["scores_sha256"], (name, q, kern)
            assert int(best[q]) == ref[q]["best_state"], (name, q, int(best[q]), ref[q]["best_state"])
        batch.close()
    forced.close()
    pbatch = model.batch(emit3, paths=True)
    pbatch.run()
    ps, pb, paths = pbatch.read(want_paths=True)
    assert pbatch.fallbacks() == 0
    for q in range(len(emit3)):
        assert sha(ps[q], np.float32) == ref[q]["scores_sha256"], (name, q, "paths run")
        assert sha(paths[q], np.int32) == ref[q]["path_sha256"], (name, q, "path")
    pbatch.close()
    model.close()


@pytest.mark.parametrize("name", MODELS)
def test_scope_spec_level2(name, scope, emit3):
    """_spec level 2 on every emit_3 row (GraphBLAS_spec_impl(2), the reference's second spec
    implementation in test_semantic_equality.cpp:46-47), bit-exact with the oracle's level-2 digests."""
    hmm = svh.read_HMM(chmm(name))
    ref = scope["models"][name]
    impl = svh.HIP_spec_impl(2)
    impl.spec_with(hmm)
    scores = impl.run_Viterbi_spec_batch(emit3)
    for q in range(len(emit3)):
        assert sha(scores[q], np.float32) == ref[q]["spec2_sha256"], (name, q)


def test_two_headline_batches_on_two_streams():
    """Two 50-sequence headline batches of one model launched back to back on two streams: 500
    workgroups of the latency plan (per-class tickets, x.xmap) against 256 CUs, so the second
    launch's workgroups wait for CUs the first holds.  Both must be bit-exact, with no fault word
    and no fallback row."""
    import torch

    hmm = svh.read_HMM(chmm("2405.chmm"))
    seqs = svh.read_emit_seq(ess("emit_50_3500_20.ess"))
    ref = load_digests()["2405.chmm x emit_50_3500_20.ess"]
    model = svh.DeviceModel(hmm, kernel=_lib.SVH_KERNEL_PIPE)  # (AUTO: the diagonal plan, test_diag_gpu.py)
    a, b = model.batch(seqs), model.batch(seqs)
    assert a.plan()["kernel"] == _lib.SVH_KERNEL_PIPE and a.plan()["pipe_groups"] == 5
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    for _ in range(3):
        a.run(0, sa.cuda_stream)
        b.run(0, sb.cuda_stream)
        for batch, st in ((a, sa), (b, sb)):
            scores, best = batch.read(st.cuda_stream)  # raises on a fault word
            assert batch.fallbacks() == 0
            for q in range(len(seqs)):
                assert sha(scores[q], np.float32) == ref[q]["scores_sha256"], q
                assert int(best[q]) == ref[q]["best_state"], q
    a.close()
    b.close()
    model.close()
