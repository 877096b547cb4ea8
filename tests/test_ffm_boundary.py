"""The Panama-FFM boundary, machine-checked without a JDK.

The Java plugin binds libosknn through hand-written `FunctionDescriptor`s
(`java/plugin/src/main/java/org/opensearch/knn/gpu/OsKnn.java`), and the Python mirror through the ctypes table
`opensearch_amd/_lib.py` `SIGNATURES`.  Nothing in this image compiles the Java side, so this test parses both
against the prototypes of `include/osknn.h` — name, arity, return type and every parameter's width:

    int32_t / uint32_t → JAVA_INT      int64_t / uint64_t → JAVA_LONG      float → JAVA_FLOAT
    double → JAVA_DOUBLE               any pointer → ADDRESS                void return → ofVoid

A descriptor that drifts from the header (an int where the C side takes int64_t, a missing argument) would
corrupt the downcall's registers at run time; here it fails on CPU.  The plugin's native access is granted the
way OpenSearch plugins get it (`--enable-native-access`, reference `build.gradle:412-415`; extension point
`server/src/main/java/org/opensearch/plugins/EnginePlugin.java:87`).
"""
import ctypes as C
import re
from pathlib import Path

import pytest

from opensearch_amd import _lib

ROOT = Path(__file__).resolve().parent.parent
HEADER = ROOT / "include" / "osknn.h"
OSKNN_JAVA = ROOT / "java" / "plugin" / "src" / "main" / "java" / "org" / "opensearch" / "knn" / "gpu" / "OsKnn.java"

_SCALAR = {"int32_t": "JAVA_INT", "uint32_t": "JAVA_INT", "int": "JAVA_INT", "int64_t": "JAVA_LONG",
           "uint64_t": "JAVA_LONG", "float": "JAVA_FLOAT", "double": "JAVA_DOUBLE", "void": "void"}


def _layout(ctype: str) -> str:
    t = ctype.strip()
    if "*" in t:
        return "ADDRESS"
    t = re.sub(r"\bconst\b", "", t).strip()
    t = t.rsplit(" ", 1)[0] if " " in t else t      # drop the parameter name
    return _SCALAR[t.strip()]


def header_prototypes(text: str | None = None) -> dict[str, tuple[str, list[str]]]:
    """name → (return layout, [parameter layouts]) for every `osk_*` function include/osknn.h declares."""
    text = HEADER.read_text() if text is None else text
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    text = re.sub(r"//[^\n]*", "", text)
    out = {}
    for m in re.finditer(r"([A-Za-z_][\w \t]*?\*?)\s*\b(osk_[a-z_0-9]+)\s*\(([^;{]*?)\)\s*;", text, flags=re.S):
        ret, name, params = m.group(1), m.group(2), " ".join(m.group(3).split())
        ret = ret.split()[-1] if "*" not in ret else "const char*"
        plist = [] if params in ("", "void") else [p.strip() for p in params.split(",")]
        out[name] = (_layout(ret if "*" in ret else ret + " r"), [_layout(p) for p in plist])
    return out


def java_descriptors(text: str) -> dict[str, tuple[str, list[str]]]:
    """name → (return layout, [parameter layouts]) of every h("osk_…", FunctionDescriptor.of…(…)) in OsKnn.java."""
    text = re.sub(r"//[^\n]*", "", text)
    out = {}
    for m in re.finditer(r'h\(\s*"(osk_[a-z_0-9]+)"\s*,\s*FunctionDescriptor\.(of|ofVoid)\(([^)]*)\)', text, flags=re.S):
        name, kind, args = m.group(1), m.group(2), [a.strip() for a in m.group(3).split(",") if a.strip()]
        args = [a.rsplit(".", 1)[-1] for a in args]          # ValueLayout.JAVA_INT → JAVA_INT
        if kind == "ofVoid":
            out[name] = ("void", args)
        else:
            out[name] = (args[0], args[1:])
    return out


def mismatches(java: dict, header: dict) -> list[str]:
    errs = []
    for name, (ret, params) in sorted(java.items()):
        if name not in header:
            errs.append(f"{name}: not declared in include/osknn.h")
            continue
        hret, hparams = header[name]
        if ret != hret:
            errs.append(f"{name}: returns {ret}, header {hret}")
        if len(params) != len(hparams):
            errs.append(f"{name}: {len(params)} parameters, header {len(hparams)}")
        for i, (a, b) in enumerate(zip(params, hparams)):
            if a != b:
                errs.append(f"{name}: parameter {i} is {a}, header {b}")
    return errs


def test_header_parser_sees_every_symbol():
    protos = header_prototypes()
    assert sorted(protos) == sorted(_lib.SIGNATURES), "parser and ctypes table disagree on the symbol set"
    assert protos["osk_seg_stage"] == ("JAVA_INT", ["JAVA_INT", "ADDRESS", "JAVA_LONG", "JAVA_INT", "JAVA_INT",
                                                    "JAVA_INT", "ADDRESS", "JAVA_INT", "ADDRESS"])
    assert protos["osk_last_error"] == ("ADDRESS", [])


def test_java_descriptors_match_the_header():
    java = java_descriptors(OSKNN_JAVA.read_text())
    assert len(java) >= 20, sorted(java)
    for needed in ("osk_seg_search", "osk_view_search", "osk_shards_search_merge", "osk_seg_stage_file",
                   "osk_comm_init_rank", "osk_topdocs_write"):
        assert needed in java
    assert mismatches(java, header_prototypes()) == []


def test_checker_fails_on_a_mismatched_descriptor():
    """The checker itself: a JAVA_INT where the header takes int64_t, a dropped argument and an unknown symbol
    are each reported."""
    text = OSKNN_JAVA.read_text()
    good = java_descriptors(text)
    bad_width = text.replace('h("osk_seg_stage", FunctionDescriptor.of(JAVA_INT,\n        JAVA_INT, ADDRESS, JAVA_LONG,',
                             'h("osk_seg_stage", FunctionDescriptor.of(JAVA_INT,\n        JAVA_INT, ADDRESS, JAVA_INT,')
    assert bad_width != text
    errs = mismatches(java_descriptors(bad_width), header_prototypes())
    assert errs == ["osk_seg_stage: parameter 2 is JAVA_INT, header JAVA_LONG"]
    bad_arity = text.replace('h("osk_seg_warm", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT))',
                             'h("osk_seg_warm", FunctionDescriptor.of(JAVA_INT, ADDRESS))')
    assert bad_arity != text
    assert mismatches(java_descriptors(bad_arity), header_prototypes()) == ["osk_seg_warm: 1 parameters, header 2"]
    extra = dict(good, osk_nope=("JAVA_INT", []))
    assert mismatches(extra, header_prototypes()) == ["osk_nope: not declared in include/osknn.h"]


_CTYPES = {C.c_int32: "JAVA_INT", C.c_uint32: "JAVA_INT", C.c_int64: "JAVA_LONG", C.c_uint64: "JAVA_LONG",
           C.c_float: "JAVA_FLOAT", C.c_double: "JAVA_DOUBLE", C.c_void_p: "ADDRESS", C.c_char_p: "ADDRESS"}


def _ctype_layout(t) -> str:
    if t in _CTYPES:
        return _CTYPES[t]
    if isinstance(t, type) and issubclass(t, C._Pointer):
        return "ADDRESS"
    raise AssertionError(f"unmapped ctypes type {t}")


@pytest.mark.parametrize("name", sorted(_lib.SIGNATURES))
def test_ctypes_table_matches_the_header(name):
    """The Python mirror's bindings (every test and the bench call through them) obey the same widths."""
    ret, args = _lib.SIGNATURES[name]
    hret, hparams = header_prototypes()[name]
    assert _ctype_layout(ret) == hret
    assert [_ctype_layout(a) for a in args] == hparams
