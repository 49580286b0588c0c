"""Keep INTEGRATION.md's reference-side code blocks equal to examples/refside/solver_bodies.cpp.

Each "<!-- body NAME -->" line in INTEGRATION.md is followed by a ```cpp block holding the text between
"// [body NAME]" and "// [end]" in solver_bodies.cpp.  `python tools/integration_bodies.py` rewrites the
blocks; tests/test_integration_doc.py checks that they are in sync (bodies() / doc_blocks())."""
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "examples", "refside", "solver_bodies.cpp")
DOC = os.path.join(ROOT, "INTEGRATION.md")
MARK = re.compile(r"<!-- body (.+?) -->\n```cpp\n(.*?)```\n", re.S)


def bodies():
    src = open(SRC).read()
    return {m.group(1): m.group(2) for m in re.finditer(r"^// \[body ([^\]\n]+)\]\n(.*?)^// \[end\]\n", src, re.S | re.M)}


def doc_blocks():
    return {m.group(1): m.group(2) for m in MARK.finditer(open(DOC).read())}


def main():
    b = bodies()
    doc = open(DOC).read()
    missing = [k for k in MARK.findall(doc) if k[0] not in b]
    if missing:
        sys.exit(f"unknown bodies: {missing}")
    doc = MARK.sub(lambda m: f"<!-- body {m.group(1)} -->\n```cpp\n{b[m.group(1)]}```\n", doc)
    open(DOC, "w").write(doc)


if __name__ == "__main__":
    main()
