"""Median kernel time of the pipelined plan (geometry from SVH_PIPE_SM / SVH_PIPE_WAVES) and a
bit-exact comparison with the serial chain kernel.  python tools/pipe_time.py MODEL ESS [REPS]"""
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
if rep > 1:
    rng = np.random.default_rng(7)
    seqs = list(seqs) + [rng.integers(0, h.emit_num, size=len(s)).astype(np.uint64) for _ in range(rep - 1) for s in seqs]
res = {}
for name, k in (("chain", _lib.SVH_KERNEL_CHAIN), ("pipe", _lib.SVH_KERNEL_PIPE)):
    m = DeviceModel(h, kernel=k)
    b = m.batch(seqs)
    b.run()
    ts = []
    for _ in range(reps):
        b.run()
        ts.append(b.elapsed_ms())
    s, bb = b.read()
    res[name] = (np.where(s == 0, 0, s), bb, float(np.median(ts)), b.plan())
eq = np.array_equal(res["chain"][0], res["pipe"][0]) and np.array_equal(res["chain"][1], res["pipe"][1])
p = res["pipe"][3]
print(f"{sys.argv[1]} x {sys.argv[2]} x{rep} SM={p['slots']} W={p['pipe_waves']} G={p['pipe_groups']}: "
      f"chain {res['chain'][2]:.3f} ms pipe {res['pipe'][2]:.3f} ms equal={eq}", flush=True)
sys.exit(0 if eq else 1)
