"""Generate the committed golden vectors (tests/golden/*.json) from the CPU oracle.

The oracle (oracle/viterbi_oracle.c) restates GraphBLAS_impl / GraphBLAS_spec_impl and is pinned
by the reference's own fixtures (tests/test_helper.h:17-22) -- see tests/test_oracle_golden.py.
Floats are stored as IEEE-754 bit patterns (hex) so the vectors are exact.

    python tests/golden/make_golden.py            # the fixture files below
    python tests/golden/make_golden.py digests    # score_digests.json (bench workloads)
    python tests/golden/make_golden.py spec2      # + level-2 digests of every emit_50 row (config 4)
    python tests/golden/make_golden.py scope      # scope_digests.json: every .chmm x emit_3_3500_20
    python tests/golden/make_golden.py sweep2     # sweep2_digests.json: level 2 of the sweep's other files
"""
from __future__ import annotations

import json
import os
import struct
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import spec_viterbi_amd as svh  # noqa: E402  (native reader only; no GPU needed)
from oracle import oracle  # noqa: E402

DATA = os.path.join(ROOT, "data")
OUT = os.path.dirname(os.path.abspath(__file__))


def hexbits(a) -> list[str]:
    return [struct.pack("<f", float(x)).hex() for x in np.asarray(a, np.float32).ravel()]


def case(hmm_path, ess_path, seq_ids, levels=(), paths=True):
    hmm = svh.read_HMM(os.path.join(DATA, hmm_path))
    seqs = svh.read_emit_seq(os.path.join(DATA, ess_path))
    out = {"chmm": hmm_path, "ess": ess_path, "sequences": []}
    for q in seq_ids:
        seq = seqs[q]
        rec = {"index": q, "length": int(seq.size)}
        if paths:
            scores, best, path = oracle.decode(hmm, seq)
            rec["best_state"] = best
            rec["path"] = path.tolist()
        else:
            scores = oracle.viterbi(hmm, seq)
        rec["scores"] = hexbits(scores)
        rec["spec"] = {str(L): hexbits(oracle.viterbi_spec(hmm, L, seq)) for L in levels}
        out["sequences"].append(rec)
    return out


def digests():
    """Per-row SHA-256 digests of the exact float32 score bytes (and of the int32 decoded paths)
    plus best states, for every sequence of the bench workloads: 2405.chmm x emit_50_3500_20
    (configs[2]), x covid-19 (configs[4]) and 100.chmm x emit_3_3500_20 (configs[1]).  bench.py checks every rank's timed output (and the
    gathered rows of its strong-scaling modes) against these without running the oracle."""
    import hashlib

    out = {}
    # (model, file): the headline and config-5 workloads, and config 2 (100.chmm x emit_3_3500_20)
    for model, ess in (("2405.chmm", "emit_50_3500_20.ess"), ("2405.chmm", "covid-19.ess"),
                       ("100.chmm", "emit_3_3500_20.ess")):
        hmm = svh.read_HMM(os.path.join(DATA, "chmm_files", model))
        seqs = svh.read_emit_seq(os.path.join(DATA, "ess_files", ess))
        rows = []
        for seq in seqs:
            scores, best, path = oracle.decode(hmm, seq)
            rows.append({"length": int(seq.size), "best_state": int(best),
                         "scores_sha256": hashlib.sha256(np.asarray(scores, np.float32).tobytes()).hexdigest(),
                         "path_sha256": hashlib.sha256(np.asarray(path, np.int32).tobytes()).hexdigest()})
        out[f"{model} x {ess}"] = rows
        print("digests", model, ess, len(rows))
    path = os.path.join(OUT, "score_digests.json")
    if os.path.exists(path):  # keep the level-2 rows (spec2_digests) in the same file
        with open(path) as f:
            out = {**json.load(f), **out}
    with open(path, "w") as f:
        json.dump(out, f, indent=0)


SPEC2_KEY = "2405.chmm x emit_50_3500_20.ess level 2"


def spec2_digests():
    """Level-2 (_spec) score digests of all 50 rows of 2405.chmm x emit_50_3500_20 (BASELINE
    config 4): the oracle builds the 400 dense products once (9.3 GB) and runs every row with them
    (GraphBLAS_spec_impl.cpp:50-89, 146-181).  Added to score_digests.json under SPEC2_KEY; rows 0..1
    are cross-checked against the full vectors in chmm2405_emit50.json first."""
    import hashlib

    hmm = svh.read_HMM(os.path.join(DATA, "chmm_files/2405.chmm"))
    seqs = svh.read_emit_seq(os.path.join(DATA, "ess_files/emit_50_3500_20.ess"))
    scores = oracle.viterbi_spec_batch(hmm, 2, seqs)
    with open(os.path.join(OUT, "chmm2405_emit50.json")) as f:
        g = json.load(f)
    for rec in g["sequences"]:
        assert hexbits(scores[rec["index"]]) == rec["spec"]["2"], rec["index"]
    rows = [{"length": int(s.size), "scores_sha256": hashlib.sha256(np.asarray(r, np.float32).tobytes()).hexdigest()}
            for s, r in zip(seqs, scores)]
    path = os.path.join(OUT, "score_digests.json")
    with open(path) as f:
        out = json.load(f)
    out[SPEC2_KEY] = rows
    with open(path, "w") as f:
        json.dump(out, f, indent=0)
    print("spec2 digests", len(rows))


def scope_digests():
    """The reference's semantic-equality scope (tests/test_semantic_equality.cpp:19-98): every
    .chmm x every sequence of emit_3_3500_20.ess, non-spec (scores, best state, decoded path) and
    _spec level 2 (scores; the oracle builds each model's S^2 dense products once), as SHA-256
    digests in scope_digests.json.  tests/test_reference_scope_gpu.py checks the GPU against them."""
    import glob
    import hashlib

    def sha(a, dt):
        return hashlib.sha256(np.ascontiguousarray(a, dt).tobytes()).hexdigest()

    seqs = svh.read_emit_seq(os.path.join(DATA, "ess_files/emit_3_3500_20.ess"))
    out = {}
    models = sorted(glob.glob(os.path.join(DATA, "chmm_files", "*.chmm")),
                    key=lambda f: int(os.path.basename(f).split(".")[0]))
    for f in models:
        name = os.path.basename(f)
        hmm = svh.read_HMM(f)
        rows = []
        spec2 = oracle.viterbi_spec_batch(hmm, 2, seqs)
        for q, seq in enumerate(seqs):
            scores, best, path = oracle.decode(hmm, seq)
            rows.append({"length": int(seq.size), "best_state": int(best), "scores_sha256": sha(scores, np.float32),
                         "path_sha256": sha(path, np.int32), "spec2_sha256": sha(spec2[q], np.float32)})
        out[name] = rows
        print("scope", name, flush=True)
    with open(os.path.join(OUT, "scope_digests.json"), "w") as fh:
        json.dump({"ess": "emit_3_3500_20.ess", "models": out}, fh, indent=0)


SWEEP2_DATASETS = ("emit_3_7000_20.ess", "covid-19.ess", "emit_50_3500_20.ess")


def sweep2_digests():
    """Level-2 score digests of the reference sweep's remaining cells (tools/bench_sweep.py): every
    .chmm x emit_3_7000_20 / covid-19 / emit_50_3500_20 that score_digests.json does not hold, each
    model's dense products built once for all three files (one viterbi_spec_batch call).  Written
    to sweep2_digests.json as {"<model> x <ess> level 2": [sha256 per row]}; resumable (models
    already in the file are skipped)."""
    import glob
    import hashlib

    path = os.path.join(OUT, "sweep2_digests.json")
    out = {}
    if os.path.exists(path):
        with open(path) as f:
            out = json.load(f)
    with open(os.path.join(OUT, "score_digests.json")) as f:
        have = json.load(f)
    data = {d: svh.read_emit_seq(os.path.join(DATA, "ess_files", d)) for d in SWEEP2_DATASETS}
    models = sorted(glob.glob(os.path.join(DATA, "chmm_files", "*.chmm")),
                    key=lambda f: int(os.path.basename(f).split(".")[0]))
    for f in models:
        name = os.path.basename(f)
        todo = [d for d in SWEEP2_DATASETS
                if f"{name} x {d} level 2" not in have and f"{name} x {d} level 2" not in out]
        if not todo:
            continue
        hmm = svh.read_HMM(f)
        seqs = [s for d in todo for s in data[d]]
        scores = oracle.viterbi_spec_batch(hmm, 2, seqs)
        k = 0
        for d in todo:
            rows = []
            for _ in data[d]:
                rows.append(hashlib.sha256(np.ascontiguousarray(scores[k], np.float32).tobytes()).hexdigest())
                k += 1
            out[f"{name} x {d} level 2"] = rows
        with open(path, "w") as fh:
            json.dump(out, fh, indent=0)
        print("sweep2", name, flush=True)


def main():
    if sys.argv[1:] == ["scope"]:
        scope_digests()
        return
    if sys.argv[1:] == ["sweep2"]:
        sweep2_digests()
        return
    if sys.argv[1:] == ["digests"]:
        digests()
        return
    if sys.argv[1:] == ["spec2"]:
        spec2_digests()
        return
    goldens = {
        "test_chmms": [case(f"chmm_files/test_chmms/{i}_test_chmm.chmm", f"ess_files/test_sequences/{i}_test_seq.ess",
                            range(2 if i == 0 else 1), levels=(1, 2, 3)) for i in range(4)],
        "chmm100_emit3": case("chmm_files/100.chmm", "ess_files/emit_3_3500_20.ess", range(3), levels=(2,)),
        "chmm2405_emit50": case("chmm_files/2405.chmm", "ess_files/emit_50_3500_20.ess", range(2), levels=(2,)),
    }
    for name, val in goldens.items():
        with open(os.path.join(OUT, f"{name}.json"), "w") as f:
            json.dump(val, f, separators=(",", ":"))
        print("wrote", name)


if __name__ == "__main__":
    main()
