"""The public headers as a C and a C++ consumer sees them.

A C99 translation unit and a C++17 one include every header under include/, take the address of every declared
entry point (so the program only links if liblo_icp.so exports them all) and print sizeof / offsetof of every
public struct.  Those layouts must equal the hand-written ctypes mirrors in lidar_odometry_amd/_lib.py, which
the Python host side and the tests pass across the ABI.  No GPU call is made (the program only loads the library).
"""
import json
import os
import shutil
import subprocess

import pytest

from lidar_odometry_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INC = os.path.join(ROOT, "include")
LIBDIR = os.path.dirname(_lib.LIB_PATH)

STRUCTS = {
    "lo_config": _lib.LoConfig,
    "lo_iter_log": _lib.LoIterLog,
    "lo_stats": _lib.LoStats,
    "lo_batch_rec": _lib.LoBatchRec,
    "lo_odom_config": _lib.LoOdomConfig,
    "lo_odom_frame": _lib.LoOdomFrame,
}


def _source():
    heads = sorted(h for h in os.listdir(INC) if h.endswith(".h"))
    lines = [f'#include "{h}"' for h in heads] + ["#include <stdio.h>", "#include <stddef.h>", ""]
    syms = sorted(_lib.EXPORTED_SYMBOLS)
    lines.append("typedef void (*any_fn)(void);")
    lines.append("static any_fn const entry_points[] = {")
    lines += [f"    (any_fn)&{s}," for s in syms]
    lines.append("};")
    lines.append("int main(void) {")
    lines.append('    printf("{\\"n_entry\\": %d", (int)(sizeof(entry_points) / sizeof(entry_points[0])));')
    for name, cls in STRUCTS.items():
        lines.append(f'    printf(", \\"{name}\\": {{\\"size\\": %d", (int)sizeof({name}));')
        for fname, _ in cls._fields_:
            lines.append(f'    printf(", \\"{fname}\\": %d", (int)offsetof({name}, {fname}));')
        lines.append('    printf("}");')
    lines.append('    printf("}\\n");')
    lines.append("    return entry_points[0] == 0;")
    lines.append("}")
    return "\n".join(lines) + "\n"


@pytest.mark.parametrize("lang", ["c", "c++"])
def test_headers_compile_link_and_match_ctypes(tmp_path, lang):
    cc = shutil.which("gcc" if lang == "c" else "g++")
    if cc is None:
        pytest.skip("no host compiler")
    if not os.path.exists(_lib.LIB_PATH):
        pytest.fail(f"{_lib.LIB_PATH} missing (build first)")
    src = tmp_path / ("abi.c" if lang == "c" else "abi.cpp")
    src.write_text(_source())
    exe = tmp_path / "abi"
    std = ["-std=c99"] if lang == "c" else ["-std=c++17"]
    cmd = [cc, *std, "-Wall", "-Wextra", "-Werror", "-pedantic", "-I", INC, str(src), "-o", str(exe),
           "-L", LIBDIR, "-llo_icp", f"-Wl,-rpath,{LIBDIR}", "-Wl,--allow-shlib-undefined"]
    p = subprocess.run(cmd, capture_output=True, text=True)
    assert p.returncode == 0, p.stderr[-3000:]
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    got = json.loads(r.stdout)
    assert got["n_entry"] == len(_lib.EXPORTED_SYMBOLS)
    for name, cls in STRUCTS.items():
        want = {"size": C_sizeof(cls), **{f: getattr(cls, f).offset for f, _ in cls._fields_}}
        assert got[name] == want, (name, got[name], want)


def C_sizeof(cls):
    import ctypes
    return ctypes.sizeof(cls)
