"""The C++ host mirror (include/syzsig_cover.hpp) compiles against the C-ABI,
and on the GPU runs pkg/cover/cover_test.go's tests (tests/cpp/cover_test.cc)."""
import os
import subprocess

import pytest

from tests.conftest import ROOT


def _kats_txt(kats, path):
    with open(path, "w") as f:
        for name, t in kats.items():
            if name == "TestMinimize":
                for c in t["cases"]:
                    covs = ";".join(" ".join(map(str, x)) for x in c["inp"])
                    f.write(f"TestMinimize 0 0|{covs}|{' '.join(map(str, c['out']))}\n")
                continue
            for c in t["cases"]:
                f.write(f"{name} {int(t['sorted'])} {int(t['symmetric'])}|{' '.join(map(str, c['v0']))}|"
                        f"{' '.join(map(str, c['v1']))}|{' '.join(map(str, c['r']))}\n")


def build_cpp_test(out_dir):
    exe = os.path.join(out_dir, "cover_test")
    lib_dir = os.path.join(ROOT, "syzkaller_amd")
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), "-o", exe,
                    os.path.join(ROOT, "tests", "cpp", "cover_test.cc"), "-L", lib_dir, "-lsyzsig",
                    f"-Wl,-rpath,{lib_dir}", "-Wl,-rpath-link,/opt/rocm/lib"], check=True)
    return exe


def test_cpp_mirror_compiles(tmp_path):
    assert os.path.exists(build_cpp_test(str(tmp_path)))


@pytest.mark.gpu
def test_cpp_cover_test_on_gpu(tmp_path, kats):
    exe = build_cpp_test(str(tmp_path))
    txt = str(tmp_path / "kats.txt")
    _kats_txt(kats, txt)
    r = subprocess.run([exe, txt], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "PASS" in r.stdout
