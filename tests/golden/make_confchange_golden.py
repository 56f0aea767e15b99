#!/usr/bin/env python3
"""Write tests/golden/confchange_datadriven.json from the reference's
TestConfChangeDataDriven data (raft/confchange/testdata/*.txt, harness
raft/confchange/datadriven_test.go:28-109).

Each file is one tracker evolving through its commands (LastIndex starts at 0
and increments after every command).  A case keeps the command, its
arguments (autoleave=...), the input line (conf change tokens) and the full
expected output text.  The datadriven text format
(github.com/cockroachdb/datadriven @ v0.0.0-20200714090401-bf6692d28da5, not
vendored) is: '#' comments, a command line, input lines, '----', the expected
output up to the next blank line.  Run here (where /root/reference exists);
the JSON is committed and is all the tests read.
"""
import glob
import json
import os

REF = "/root/reference/raft/confchange/testdata"
HERE = os.path.dirname(os.path.abspath(__file__))


def parse(path):
    lines = open(path, encoding="utf-8").read().split("\n")
    cases, i = [], 0
    while i < len(lines):
        ln = lines[i]
        if ln.strip() == "" or ln.startswith("#"):
            i += 1
            continue
        cmdline, line_no = ln, i + 1
        i += 1
        inp = []
        while lines[i] != "----":
            inp.append(lines[i])
            i += 1
        i += 1
        out = []
        while i < len(lines) and lines[i] != "":
            out.append(lines[i])
            i += 1
        parts = cmdline.split()
        case = {"file": os.path.basename(path), "line": line_no, "cmd": parts[0],
                "input": " ".join(inp), "expected": "\n".join(out) + "\n"}
        for a in parts[1:]:
            k, v = a.split("=")
            assert k == "autoleave"
            case["autoleave"] = v == "true"
        cases.append(case)
    return cases


def main():
    files = {}
    for p in sorted(glob.glob(os.path.join(REF, "*.txt"))):
        files[os.path.basename(p)] = parse(p)
    with open(os.path.join(HERE, "confchange_datadriven.json"), "w", encoding="utf-8") as f:
        json.dump(files, f, indent=1)
    print(sum(len(v) for v in files.values()), "cases in", len(files), "files")


if __name__ == "__main__":
    main()
