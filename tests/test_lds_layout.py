"""The sweeps' LDS carves are compile-time layouts (dpe-mvs_amd/csrc/lds_layout.h): every region of
the strong sweep's per-wave block and the weak sweep's per-pixel block is checked by static_assert for
bounds, alignment and pairwise overlap at every source-view count 1..31, plus the LDS budgets.  Here:
the header compiles (its asserts hold), and a deliberately overlapping layout does not."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "dpe-mvs_amd", "csrc", "lds_layout.h")


def _compile(tmp_path, body):
    src = tmp_path / "t.cpp"
    src.write_text(f'#include "{HDR}"\n{body}\nint main() {{ return 0; }}\n')
    return subprocess.run(["g++", "-std=c++17", "-fsyntax-only", str(src)], capture_output=True, text=True)


def test_layouts_hold(tmp_path):
    r = _compile(tmp_path, "static_assert(dpe::lds::StrongCarve<4, 16, 16>::total(9) == 1652 + 4 * 17 * 5 + 288 + 4 * 12, \"\");\n"
                           "static_assert(dpe::lds::WeakCarve::per_pixel(9) == 636, \"\");")
    assert r.returncode == 0, r.stderr


def test_overlapping_layout_does_not_compile(tmp_path):
    # a region that runs one float into its neighbour (the kind of carve error that faulted the GPU
    # in round 3: a row-sum buffer overlapping a job list)
    bad = ("constexpr dpe::lds::Region r[] = {{0, 108, 1}, {107, 72, 1}};\n"
           "static_assert(dpe::lds::regions_ok(r, 400), \"overlap\");")
    r = _compile(tmp_path, bad)
    assert r.returncode != 0 and "overlap" in r.stderr
    misaligned = ("constexpr dpe::lds::Region r[] = {{0, 10, 1}, {10, 32, 4}};\n"
                  "static_assert(dpe::lds::regions_ok(r, 400), \"align\");")
    r = _compile(tmp_path, misaligned)
    assert r.returncode != 0 and "align" in r.stderr
    good = "constexpr dpe::lds::Region r[] = {{0, 108, 1}, {108, 72, 1}};\nstatic_assert(dpe::lds::regions_ok(r, 400), \"\");"
    assert _compile(tmp_path, good).returncode == 0
