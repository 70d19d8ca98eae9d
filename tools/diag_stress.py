"""Stress check of the diagonal plan: the headline batch and a fallback-heavy model, many passes on
one batch; prints per pass the rows that differ from the reference (digests / oracle) and the
fallback rows."""
import hashlib
import sys
import numpy as np
sys.path.insert(0, ".")
import spec_viterbi_amd as svh
from spec_viterbi_amd import _lib
from oracle import oracle
from tests.conftest import chmm, ess
from tests.helpers import random_chain_hmm, random_seqs, bit_equal, load_digests

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
hmm = svh.read_HMM(chmm("2405.chmm"))
seqs = svh.read_emit_seq(ess("emit_50_3500_20.ess"))
rows = load_digests()["2405.chmm x emit_50_3500_20.ess"]
m = svh.DeviceModel(hmm)
b = m.batch(seqs)
bad_total = 0
for r in range(reps):
    b.run()
    s, best = b.read()
    bad = [q for q in range(len(seqs)) if hashlib.sha256(np.ascontiguousarray(s[q]).tobytes()).hexdigest() != rows[q]["scores_sha256"]]
    fr = np.nonzero(b.fallback_rows())[0].tolist()
    bad_total += len(bad)
    if bad or fr:
        print("headline pass", r, "bad", bad, "fallback", fr, flush=True)
print("headline bad rows total", bad_total, flush=True)
hmm = random_chain_hmm(600, S=12, seed=11, self_n=False)
seqs = random_seqs(12, [300, 64, 1, 97, 33], seed=12)
refs, _ = oracle.viterbi_batch(hmm, seqs)
m = svh.DeviceModel(hmm, kernel=_lib.SVH_KERNEL_DIAG)
b = m.batch(seqs)
bad_total = 0
for r in range(reps):
    b.run()
    s, best = b.read()
    bad = [q for q in range(len(seqs)) if not bit_equal(s[q], refs[q])]
    bad_total += len(bad)
    if bad:
        print("variant0 pass", r, "bad", bad, "fallback", np.nonzero(b.fallback_rows())[0].tolist(), flush=True)
print("variant0 bad rows total", bad_total, flush=True)
