"""The drop-in boundary compiles into the reference application.

The reference app includes the renderer header and its own GL SSAO class side by side
(/root/reference/sphereflake/main.cpp:71-72; SSAO.h:6-50 defines SphereflakeRaytracer::SSAO). This test
copies main.cpp into a temporary directory at test time (it is never committed), applies exactly the edits
INTEGRATION.md §2 prints -- the include swap with SF_USE_GLM and the one added Render() line in
SphereflakeRaytracerMain::Render (main.cpp:301-304) -- and syntax-compiles it with g++ against the
reference's own glm / GLFW headers and this repository's Sphereflake.hpp. It also checks that INTEGRATION.md
quotes the same edits, so the documented patch and the tested patch cannot drift apart.

Skipped where /root/reference is absent (the GPU box).
"""
import os
import pathlib
import shutil
import subprocess

import pytest

REF = pathlib.Path("/root/reference")
ROOT = pathlib.Path(__file__).resolve().parents[1]
CSRC = ROOT / "sphereflake-raytracer_amd" / "csrc"

# INTEGRATION.md §2, edit 1: the include swap (main.cpp:71)
INCLUDE_OLD = '#include "Sphereflake.h"\n'
INCLUDE_NEW = '#define SF_USE_GLM\n#include "Sphereflake.hpp"          // was: #include "Sphereflake.h"\n'
# INTEGRATION.md §2, edit 2: one full frame after the per-frame SetView (main.cpp:304)
SETVIEW = ("m_Sphereflake.SetView(m_Camera->GetPosition(), m_Camera->GetTopLeft(), "
           "m_Camera->GetTopRight(), m_Camera->GetBottomLeft());\n")
RENDER_LINE = "m_Sphereflake.Render();"

pytestmark = pytest.mark.skipif(not (REF / "sphereflake" / "main.cpp").exists(),
                                reason="reference tree not present")


def _patched_main(src: str) -> str:
    assert src.count(INCLUDE_OLD) == 1
    src = src.replace(INCLUDE_OLD, INCLUDE_NEW)
    # the per-frame SetView inside Render() is the one followed by the positions PBO upload (main.cpp:304-306)
    marker = SETVIEW + "\n\t\tm_PositionsPbo"
    assert src.count(marker) == 1
    return src.replace(marker, SETVIEW + "\t\t" + RENDER_LINE + "\n\n\t\tm_PositionsPbo")


def _compile(path: pathlib.Path) -> subprocess.CompletedProcess:
    inc = [REF / "sphereflake", REF / "lib" / "glm" / "glm", REF / "lib" / "glfw" / "include",
           ROOT / "include", CSRC]
    cmd = ["g++", "-std=c++17", "-fsyntax-only", "-mavx"] + [f"-I{p}" for p in inc] + [str(path)]
    return subprocess.run(cmd, capture_output=True, text=True, timeout=300)


def test_patched_reference_main_compiles(tmp_path):
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    main = tmp_path / "main.cpp"
    main.write_text(_patched_main((REF / "sphereflake" / "main.cpp").read_text()))
    # nothing else in the temp dir: Sphereflake.hpp must come from csrc/, the rest from the reference tree
    assert sorted(os.listdir(tmp_path)) == ["main.cpp"]
    r = _compile(main)
    assert r.returncode == 0, r.stderr[-4000:]


def test_drop_in_header_defines_no_reference_ssao():
    """The headless SSAO lives in SphereflakeSSAO.hpp, namespace Headless: Sphereflake.hpp itself must not
    define a class SSAO, which is what broke the round-4 patch (redefinition of SphereflakeRaytracer::SSAO)."""
    hpp = (CSRC / "Sphereflake.hpp").read_text()
    assert "class SSAO" not in hpp
    ssao = (CSRC / "SphereflakeSSAO.hpp").read_text()
    assert "namespace Headless" in ssao and "class SSAO" in ssao


def test_integration_doc_quotes_the_tested_edits():
    doc = (ROOT / "INTEGRATION.md").read_text()
    assert INCLUDE_NEW.strip() in doc
    assert RENDER_LINE in doc
    assert SETVIEW.split("(")[0] in doc


LIB = ROOT / "sphereflake-raytracer_amd" / "build" / "libsphereflake_hip.so"


def _object(path: pathlib.Path, out: pathlib.Path, extra_inc=()) -> subprocess.CompletedProcess:
    inc = list(extra_inc) + [REF / "sphereflake", REF / "lib" / "glm" / "glm", REF / "lib" / "glfw" / "include",
                             ROOT / "include", CSRC]
    cmd = ["g++", "-std=c++17", "-c", "-O1", "-mavx"] + [f"-I{p}" for p in inc] + [str(path), "-o", str(out)]
    return subprocess.run(cmd, capture_output=True, text=True, timeout=300)


def _symbols(args) -> set:
    r = subprocess.run(["nm"] + args, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    return {line.split()[-1] for line in r.stdout.splitlines() if line.strip()}


def _demangle(names) -> dict:
    names = sorted(names)
    r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True, timeout=60)
    return dict(zip(names, r.stdout.splitlines()))


def unresolved_drop_in_symbols(obj: pathlib.Path, lib: pathlib.Path) -> list:
    """The drop-in symbols the object needs -- SphereflakeRaytracer::Sphereflake::* (the class members) and the sf_*
    C ABI -- that the library does not define (demangled). main.cpp's GL and SSAO classes are the reference's own
    translation units, linked beside it, and are not the drop-in's."""
    need = _symbols(["-u", str(obj)])
    have = _symbols(["-D", "--defined-only", str(lib)])
    dem = _demangle(need)
    ours = [n for n in need if dem[n].startswith("SphereflakeRaytracer::Sphereflake::") or n.startswith("sf_")]
    return sorted(dem[n] for n in ours if n not in have)


def test_patched_reference_main_links_against_the_library(tmp_path):
    """the patched reference main.cpp compiled to an object (not just syntax-checked), and every
    SphereflakeRaytracer::Sphereflake member / sf_* function it references is exported by libsphereflake_hip.so.
    A negative control proves the check bites: a member declared in a copy of the header but defined nowhere."""
    if shutil.which("g++") is None or shutil.which("nm") is None:
        pytest.skip("binutils / g++ not available")
    if not LIB.exists():
        pytest.skip("library not built (make -C sphereflake-raytracer_amd)")
    main = tmp_path / "main.cpp"
    main.write_text(_patched_main((REF / "sphereflake" / "main.cpp").read_text()))
    obj = tmp_path / "main.o"
    r = _object(main, obj)
    assert r.returncode == 0, r.stderr[-4000:]
    dem = _demangle(_symbols(["-u", str(obj)]))
    used = {d for d in dem.values() if d.startswith("SphereflakeRaytracer::Sphereflake::")}
    # the exported members behind what main.cpp calls: the ctor (Open), SetView (SetViewFloats), Render, GetGBuffer
    # (Refresh), the stats getters/resetters, the dtor (Close) -- the vector-typed members are inline in the header
    for member in ("Open(", "SetViewFloats(", "Render(", "Refresh(", "Close(", "GetClosestSphereDistance(",
                   "GetMaxDepthReached(", "ResetRaysPerSecond("):
        assert any(member in d for d in used), (member, sorted(used))
    assert unresolved_drop_in_symbols(obj, LIB) == []
    # negative control
    hdr = tmp_path / "inc"
    hdr.mkdir()
    text = (CSRC / "Sphereflake.hpp").read_text()
    anchor = "void Render(const sf_render_params* params = nullptr);"
    assert text.count(anchor) == 1, "Sphereflake.hpp declares Render()"
    (hdr / "Sphereflake.hpp").write_text(text.replace(anchor, anchor + " void NotExported();", 1))
    probe = tmp_path / "probe.cpp"
    probe.write_text('#include "Sphereflake.hpp"\n'
                     "void f(SphereflakeRaytracer::Sphereflake& s) { s.Render(); s.NotExported(); }\n")
    pobj = tmp_path / "probe.o"
    r = _object(probe, pobj, extra_inc=[hdr])
    assert r.returncode == 0, r.stderr[-4000:]
    missing = unresolved_drop_in_symbols(pobj, LIB)
    assert missing == ["SphereflakeRaytracer::Sphereflake::NotExported()"], missing
