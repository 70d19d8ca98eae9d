import sys, numpy as np
sys.path.insert(0, '.')
import spec_viterbi_amd as svh
from oracle import oracle
from tests.helpers import random_chain_hmm, random_seqs
hmm = random_chain_hmm(700, seed=6)
seqs = random_seqs(20, [1, 2, 3, 4, 5, 6, 7, 8, 9, 63, 64, 65, 77, 1000, 5000], seed=6)
m = svh.DeviceModel(hmm)
print(m.info())
for q in [9, 10, 11, 12, 13]:
    seq = seqs[q]
    sc, best, pth = m.viterbi([seq], paths=True)
    ref, rb, rp = oracle.decode(hmm, seq)
    bad = np.nonzero(pth[0] != rp)[0]
    print(q, len(seq), 'mismatch at', bad[:8])
    if bad.size:
        _, bp = oracle.viterbi(hmm, seq, backpointers=True)
        t = bad[-1]  # last mismatching obs; its successor state is shared
        s_next = rp[t + 1]
        print('  obs', t + 1, 'state', s_next, 'ref pred', bp[t, s_next], 'gpu pred', pth[0][t])
        v = oracle.viterbi(hmm, seq[:t + 1])
        o = int(seq[t + 1]); E = hmm.emissions[o]
        r = hmm.trans_rows; c = hmm.trans_cols; p = hmm.trans_probs
        for k in np.nonzero(c == s_next)[0]:
            src = int(r[k]); term = np.float32(np.float32(E[s_next] + p[k]) + v[src])
            print('   term from', src, repr(term))
