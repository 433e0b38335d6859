#!/usr/bin/env python3
"""Regenerate the golden fixtures under tests/golden/ from the reference's own data files.

Run in the build container (the only place /root/reference exists):

    python tests/golden/make_golden.py [/root/reference]

What it writes (all DATA — inputs and expected outputs the reference already holds):

* ``fasta/*.fa``           byte-for-byte copies of the reference FASTA inputs
                            (``data/query1.fa``, ``data/query100.fa``, ``data/data{1,10,20,40,60,100,500}.fa``).
* ``ref_scores.tsv``       one row per golden pair: source, library, query, target name, score.
    - source ``hdl``       ScoreBank ModelSim transcripts ``data/<lib>_<query>_out.txt``
                            (written by ``ScoreBank/ScoreBank_v1_tb.sv:271-285``; S = biased - 2048).
    - source ``ssearch36`` ``data/score.txt`` / ``data/score500.txt`` column 6
                            (``ssearch36 -3 -R``, ``data/ssearch36_command:6``; params at ``data/score500.txt:503``).
    - source ``capi``      ``capi_sample_aligner/software-C,C++/build/main_test_output.txt`` (``result: 102``),
                            query1 vs the first library record the CAPI host read (``data1.fa`` db18, 128 bp).
* ``swalign_control.tsv``  ``data/sw_testing.txt`` scores (swalign, gap = go+(k-1)*ge): a NEGATIVE control
                            (``data/sw-testing.py:31-36``); 4 of its 16 scores must differ from ours.
* ``score500_R_lines.txt``  the 499 per-target lines of ``data/score500.txt`` verbatim (ssearch36 ``-R``
                            layout: name, length, score, record index, byte offset), to check the CLI's
                            ``-R`` writer byte for byte.
* ``charto2bit_query1.hex`` the 2-bit packing the CAPI host printed for query1
                            (``build/main_test_output.txt`` "data[k]: 0x.." lines).

Nothing from the reference's source code is copied; transcripts are parsed into plain tables.
"""
import os
import re
import shutil
import sys

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
DATA = os.path.join(REF, "data")

FASTA = ["query1.fa", "query100.fa", "data1.fa", "data10.fa", "data20.fa", "data40.fa",
         "data60.fa", "data100.fa", "data500.fa"]

TRANSCRIPTS = [  # (library, query) -> data/<lib>_<query>_out.txt
    ("data1.fa", "query1.fa"), ("data10.fa", "query1.fa"), ("data10.fa", "query100.fa"),
    ("data20.fa", "query100.fa"), ("data40.fa", "query100.fa"), ("data60.fa", "query100.fa"),
    ("data100.fa", "query100.fa"), ("data500.fa", "query100.fa"),
]
SSEARCH = [("score.txt", "data100.fa", "query100.fa"), ("score500.txt", "data500.fa", "query100.fa")]

LINE_RE = re.compile(r"^@\s*\d+ns:\s+>(\S+)\s+score:\s+(-?\d+)\s*$")


def main():
    os.makedirs(os.path.join(HERE, "fasta"), exist_ok=True)
    for f in FASTA:
        shutil.copyfile(os.path.join(DATA, f), os.path.join(HERE, "fasta", f))

    rows = []
    for lib, q in TRANSCRIPTS:
        path = os.path.join(DATA, f"{lib}_{q}_out.txt")
        for line in open(path):
            m = LINE_RE.match(line.rstrip("\n"))
            if m:
                rows.append(("hdl", lib, q, m.group(1), int(m.group(2))))
    for fname, lib, q in SSEARCH:
        for line in open(os.path.join(DATA, fname)):
            tok = line.split()
            if len(tok) >= 6 and tok[0].startswith("db") and tok[1].isdigit():
                rows.append(("ssearch36", lib, q, tok[0], int(tok[5])))

    with open(os.path.join(HERE, "score500_R_lines.txt"), "w") as out:
        for line in open(os.path.join(DATA, "score500.txt")):
            if line.startswith("db"):
                out.write(line.rstrip("\n") + "\n")

    capi_out = os.path.join(REF, "capi_sample_aligner", "software-C,C++", "build", "main_test_output.txt")
    txt = open(capi_out, errors="replace").read()
    m = re.search(r"result:\s*(-?\d+),\s*biased:\s*(\d+)", txt)
    rows.append(("capi", "data1.fa", "query1.fa", "db18", int(m.group(1))))

    with open(os.path.join(HERE, "ref_scores.tsv"), "w") as out:
        out.write("source\tlibrary\tquery\ttarget\tscore\n")
        for r in rows:
            out.write("\t".join(str(x) for x in r) + "\n")

    # swalign negative control (tail "dbN:\tS" lines)
    ctrl = []
    for line in open(os.path.join(DATA, "sw_testing.txt")):
        m = re.match(r"^(db\d+):\t(-?\d+)$", line.rstrip("\n"))
        if m:
            ctrl.append((m.group(1), int(m.group(2))))
    with open(os.path.join(HERE, "swalign_control.tsv"), "w") as out:
        out.write("library\tquery\ttarget\tscore\n")
        for name, s in ctrl:
            out.write(f"data1.fa\tquery1.fa\t{name}\t{s}\n")

    # charTo2bit bytes for query1 as printed by the CAPI host (first "ID: 0000000000" block)
    blk = txt.split("ID: 0000000001")[0]
    hexes = re.findall(r"data\[\s*(\d+)\]: 0x([0-9a-f]{2})", blk)
    nbytes = 8  # 32 bases / 4 per byte; later bytes are stack garbage printed by the host
    with open(os.path.join(HERE, "charto2bit_query1.hex"), "w") as out:
        out.write(" ".join(h for _, h in hexes[:nbytes]) + "\n")
    print(f"wrote {len(rows)} golden scores, {len(ctrl)} control scores")


if __name__ == "__main__":
    main()
