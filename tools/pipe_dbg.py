"""One pipelined pass with SVH_PIPE_DEBUG counters (stderr).  python tools/pipe_dbg.py MODEL ESS"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from spec_viterbi_amd import _lib  # noqa: E402
from spec_viterbi_amd.hmm import read_emit_seq, read_HMM  # noqa: E402
from spec_viterbi_amd.viterbi import DeviceModel  # noqa: E402

root = os.path.join(os.path.dirname(__file__), "..", "data")
h = read_HMM(os.path.join(root, "chmm_files", sys.argv[1] + ".chmm"))
seqs = read_emit_seq(os.path.join(root, "ess_files", sys.argv[2] + ".ess"))
m = DeviceModel(h, kernel=_lib.SVH_KERNEL_PIPE)
b = m.batch(seqs)
for _ in range(2):
    b.run()
    print("ms", b.elapsed_ms(), flush=True)
