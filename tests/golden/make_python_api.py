"""Generate tests/golden/python_node_api.json: the reference Python `Node`'s public surface — every
method of its `#[pymethods] impl Node` block (apis/python/node/src/lib.rs:41-210) with its Python
parameters (pyo3 `signature` defaults where given), read from the reference's source text.

Run from the repo root with the reference at /root/reference:
    python tests/golden/make_python_api.py
The fixture is data (names, parameters, defaults); tests/test_python_node_api.py holds
dora_amd.node.Node to it without reading the reference.
"""
import json
import os
import re
import sys

REF = "/root/reference/apis/python/node/src/lib.rs"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "python_node_api.json")
# Rust parameters that are not Python parameters
RUST_ONLY = {"self", "&self", "&mut self", "slf", "py"}


def split_args(s: str):
    """Split a Rust parameter list at top-level commas (generics hold commas too)."""
    out, depth, cur = [], 0, ""
    for c in s:
        if c in "<(":
            depth += 1
        elif c in ">)":
            depth -= 1
        if c == "," and depth == 0:
            out.append(cur.strip())
            cur = ""
        else:
            cur += c
    if cur.strip():
        out.append(cur.strip())
    return out


def parse(txt: str) -> dict:
    start = txt.index("#[pymethods]\nimpl Node {")
    depth, i = 0, txt.index("{", start)
    end = i
    for j in range(i, len(txt)):
        if txt[j] == "{":
            depth += 1
        elif txt[j] == "}":
            depth -= 1
            if depth == 0:
                end = j
                break
    block = txt[start:end]
    methods = {}
    sig_re = re.compile(r"#\[pyo3\(signature\s*=\s*\((.*?)\)\)\]", re.S)
    for m in re.finditer(r"(?:pub\s+)?fn\s+(\w+)\s*\((.*?)\)\s*(?:->|\{)", block, re.S):
        name, rust_args = m.group(1), m.group(2)
        head = block[max(0, m.start() - 400):m.start()]
        sig = sig_re.findall(head[head.rfind("fn ") + 1 if "fn " in head else 0:])
        params = []
        for a in split_args(rust_args):
            pname = a.split(":")[0].strip()
            if pname in RUST_ONLY or a.startswith("&") or a.endswith("Python") or \
                    "PyRef<" in a:
                continue
            params.append({"name": pname, "default": None, "has_default": False})
        if sig:
            defaults = {}
            for p in split_args(sig[-1]):
                if "=" in p:
                    k, v = [y.strip() for y in p.split("=", 1)]
                    defaults[k] = v
            for p in params:
                if p["name"] in defaults:
                    p["has_default"] = True
                    p["default"] = None if defaults[p["name"]] == "None" else defaults[p["name"]]
        py_name = "__init__" if name == "new" else name
        methods[py_name] = params
    return methods


def main():
    txt = open(REF).read()
    api = {"source": "apis/python/node/src/lib.rs (#[pymethods] impl Node)",
           "methods": parse(txt)}
    with open(OUT, "w") as f:
        json.dump(api, f, indent=1, sort_keys=True)
    print(json.dumps(api, indent=1, sort_keys=True))


if __name__ == "__main__":
    sys.exit(main())
