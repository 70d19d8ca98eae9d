# Diagnostic: median time of the decoded-path batch on 2405.chmm x emit_50 (decoded-path variant + traceback).
import os, statistics, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spec_viterbi_amd as svh
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
hmm = svh.read_HMM(os.path.join(R, "data", "chmm_files", "2405.chmm"))
seqs = svh.read_emit_seq(os.path.join(R, "data", "ess_files", "emit_50_3500_20.ess"))
m = svh.DeviceModel(hmm)
b = m.batch(seqs, paths=True)
t = []
for k in range(18):
    b.run()
    if k >= 3:
        t.append(b.elapsed_ms())
print(sys.argv[1] if len(sys.argv) > 1 else "", f"median {statistics.median(t):.4f} ms min {min(t):.4f}", flush=True)
