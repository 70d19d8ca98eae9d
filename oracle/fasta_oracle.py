"""CPU restatement of the reference's FASTA -> .ess conversion (TEST INFRASTRUCTURE ONLY).

Follows ess_files/fasta_to_ess.py:3-45 of IvanTyulyandin/Spec_Viterbi line by line in behaviour:
  * amino2num (:3-7): ACDEFGHIKLMNPQRSTVWY -> 0..19, X -> 0 ("X can be transformed into any
    aminoacid"); any other residue raises KeyError (:36-37);
  * every line is stripped (:21-22); a line whose first character is '>' closes the current
    sequence if it is non-empty (:27-30); other lines extend it with their characters (:31-32);
    an empty line raises IndexError at line[0] (:27);
  * the last non-empty sequence is kept (:33-34); output: count, then "i len" and the symbols.
Only tests/ import this module, as the checker of the native reader (spec_viterbi_amd/stream.py).
"""
from __future__ import annotations

AMINO2NUM = {a: i for i, a in enumerate("ACDEFGHIKLMNPQRSTVWY")}
AMINO2NUM["X"] = 0


def fasta_sequences(text: str) -> list[list[int]]:
    """Sequences of a FASTA text as symbol lists (raises IndexError / KeyError like the script)."""
    data = [x.strip() for x in text.splitlines(keepends=True)]
    seq_list, cur = [], []
    for line in data:
        if line[0] == ">":
            if cur:
                seq_list.append(cur)
            cur = []
        else:
            cur.extend(line)
    if cur:
        seq_list.append(cur)
    return [[AMINO2NUM[a] for a in seq] for seq in seq_list]


def ess_text(seqs: list[list[int]]) -> str:
    """The .ess text fasta_to_ess.py writes (:42-45)."""
    out = [f"{len(seqs)}\n"]
    for i, seq in enumerate(seqs):
        out.append(f"{i} {len(seq)}\n" + " ".join(map(str, seq)) + "\n")
    return "".join(out)
