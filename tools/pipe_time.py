"""Median kernel time of the pipelined plans (latency geometry from SVH_PIPE_SM / SVH_PIPE_WAVES,
wide geometry from SVH_PIPEW_SM / SVH_PIPEW_WAVES) against the serial chain kernel (its wide plan
for batches of more sequences than CUs), with a bit-exact comparison.
python tools/pipe_time.py MODEL ESS [REPS] [REPLICATE] [KERNELS]   KERNELS: e.g. chain,pipe,pipew"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from spec_viterbi_amd import _lib  # noqa: E402
from spec_viterbi_amd.hmm import read_emit_seq, read_HMM  # noqa: E402
from spec_viterbi_amd.viterbi import DeviceModel  # noqa: E402

root = os.path.join(os.path.dirname(__file__), "..", "data")
h = read_HMM(os.path.join(root, "chmm_files", sys.argv[1] + ".chmm"))
seqs = read_emit_seq(os.path.join(root, "ess_files", sys.argv[2] + ".ess"))
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
rep = int(sys.argv[4]) if len(sys.argv) > 4 else 1  # copies of the file's sequences (synthetic)
names = (sys.argv[5] if len(sys.argv) > 5 else "chain,pipe").split(",")
if rep > 1:
    rng = np.random.default_rng(7)
    seqs = list(seqs) + [rng.integers(0, h.emit_num, size=len(s)).astype(np.uint64) for _ in range(rep - 1) for s in seqs]
kernels = {"chain": _lib.SVH_KERNEL_CHAIN, "pipe": _lib.SVH_KERNEL_PIPE, "pipew": _lib.SVH_KERNEL_PIPE_WIDE,
           "auto": _lib.SVH_KERNEL_AUTO}
res = {}
for name in names:
    m = DeviceModel(h, kernel=kernels[name])
    b = m.batch(seqs)
    b.run()
    ts = []
    for _ in range(reps):
        b.run()
        ts.append(b.elapsed_ms())
    s, bb = b.read()
    fb = b.fallbacks()
    res[name] = (np.where(s == 0, 0, s), bb, float(np.median(ts)), b.plan(), fb)
ref = res[names[0]]
ok = True
line = f"{sys.argv[1]} x {sys.argv[2]} x{rep} ({len(seqs)} seqs):"
for name in names:
    r = res[name]
    eq = np.array_equal(ref[0], r[0]) and np.array_equal(ref[1], r[1])
    ok &= eq
    p = r[3]
    line += (f" {name} {r[2]:.3f} ms [k{p['kernel']} {p['threads']}x{p['slots']} fb={r[4]}]"
             + ("" if eq else " DIFFERS"))
print(line, flush=True)
sys.exit(0 if ok else 1)
