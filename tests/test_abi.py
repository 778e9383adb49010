"""The C-ABI library loads and exports every entry point include/*.h declares (no GPU calls)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared(header):
    src = open(os.path.join(ROOT, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mtr_\w+)\s*\(", src)))


@pytest.fixture(scope="module")
def libmtr():
    path = os.path.join(ROOT, "fluidframework_amd", "libmtr.so")
    if not os.path.exists(path):
        from fluidframework_amd import build
        build.build_engine()
    return ctypes.CDLL(path)


def test_header_declares_the_client_surface():
    names = declared("mtr.h")
    for n in ("mtr_engine_create", "mtr_submit", "mtr_run", "mtr_summarize", "mtr_get_summary", "mtr_get_text",
              "mtr_doc_status", "mtr_engine_destroy"):
        assert n in names


def test_every_declared_symbol_is_exported(libmtr):
    missing = [n for n in declared("mtr.h") if not hasattr(libmtr, n)]
    assert not missing, f"libmtr.so lacks {missing}"


def test_library_is_gfx950_code(libmtr):
    blob = open(os.path.join(ROOT, "fluidframework_amd", "libmtr.so"), "rb").read()
    assert b"gfx950" in blob


def test_product_path_does_not_import_the_oracle():
    pkg = os.path.join(ROOT, "fluidframework_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".h", ".cc", ".cpp", ".js")):
                text = open(os.path.join(dirpath, f), errors="replace").read()
                assert "oracle" not in re.findall(r"(?:import|from|#include|require)\s*\(?\s*[\"']?([\w./]+)", text) \
                    and "liboracle" not in text, f"{f} references the oracle"
