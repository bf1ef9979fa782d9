"""CPU: the Java FFM binding in INTEGRATION.md cannot be compiled here (no
JDK), so its text is checked against the C header instead: every downcall it
declares names an exported entry point of include/tlcgpu.h, its
FunctionDescriptor has one layout per C parameter plus the return, and the
struct sizes its comments state are the C compiler's."""
import ctypes
import os
import re

import tlcgpu
from conftest import ROOT


def header_prototypes():
    """name -> (return type, [parameter types]) of every function in tlcgpu.h"""
    with open(os.path.join(ROOT, "include", "tlcgpu.h")) as f:
        text = re.sub(r"/\*.*?\*/", " ", f.read(), flags=re.S)
    protos = {}
    for ret, name, args in re.findall(r"([A-Za-z_][A-Za-z_0-9 \*]*?)\s*\b(tlcg_[a-z_0-9]+)\s*\(([^)]*)\)\s*;", text):
        params = [a.strip() for a in args.split(",") if a.strip() and a.strip() != "void"]
        protos[name] = (ret.strip(), params)
    return protos


def java_block():
    with open(os.path.join(ROOT, "INTEGRATION.md")) as f:
        text = f.read()
    m = re.search(r"```java\n(.*?)```", text, flags=re.S)
    assert m, "INTEGRATION.md has no Java block"
    return m.group(1)


def java_downcalls():
    """name -> the layouts listed in its FunctionDescriptor (return first, or
    None for ofVoid)"""
    java = re.sub(r"\s+", " ", java_block())
    out = {}
    for name, kind, body in re.findall(r'h\("(tlcg_[a-z_0-9]+)", FunctionDescriptor\.(of|ofVoid)\(([^;]*?)\)\)', java):
        layouts = [x.strip() for x in body.split(",") if x.strip()]
        out[name] = ([None] if kind == "ofVoid" else []) + layouts
    return out


def c_layout(ctype):
    t = ctype.replace("const", "").strip()
    if "*" in t:
        return "ADDRESS"
    t = t.split()[0] if t.split() else t
    return {"int": "JAVA_INT", "int32_t": "JAVA_INT", "uint64_t": "JAVA_LONG", "int64_t": "JAVA_LONG",
            "double": "JAVA_DOUBLE", "void": None}[t]


def test_java_downcalls_match_the_header():
    protos = header_prototypes()
    calls = java_downcalls()
    assert len(calls) >= 8
    for name, layouts in calls.items():
        assert name in protos, name
        ret, params = protos[name]
        want = [c_layout(ret)] + [c_layout(p.rsplit(" ", 1)[0] if not p.endswith("*") else p) for p in params]
        assert layouts == want, (name, layouts, want)


def test_java_struct_sizes_are_the_c_sizes():
    text = java_block()
    sizes = dict((n, int(b)) for n, b in re.findall(r"(tlcg_[a-z]+) (\d+) B", text))
    assert {"tlcg_model", "tlcg_opts", "tlcg_stats", "tlcg_liveness"} <= set(sizes)
    for name, size in sizes.items():
        assert ctypes.sizeof(getattr(tlcgpu, name)) == size, name
