"""C++ host mirror (include/addapt/*.hh over the C ABI) without a GPU: the
reference's model / sampling / scoring test cases restated in
tests/cpp/test_host.cc (DummyRnaFold, as the reference tests do), the
config reader and the TSV trajectory format."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "addapt_amd", "_lib")


@pytest.fixture(scope="module")
def host_lib():
    from addapt_amd import _build

    _build.build_gpu()
    _build.build_host()
    return LIB


def test_cpp_host_unit_tests(host_lib, tmp_path):
    exe = str(tmp_path / "test_host")
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-I", os.path.join(ROOT, "include"), "-o", exe,
                    os.path.join(ROOT, "tests", "cpp", "test_host.cc"), "-L", host_lib, "-laddapt_host",
                    "-laddapt_gpu", "-Wl,-rpath," + host_lib], check=True)
    r = subprocess.run([exe], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=120)
    assert r.returncode == 0, r.stdout
    assert " 0 failed" in r.stdout


def test_cli_usage(host_lib):
    exe = os.path.join(host_lib, "addapt")
    r = subprocess.run([exe, "--help"], stdout=subprocess.PIPE, text=True, timeout=60)
    assert r.returncode == 0 and "Usage:" in r.stdout and "--num-moves" in r.stdout
    r = subprocess.run([exe, "/nonexistent.yml"], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                       text=True, timeout=60)
    assert r.returncode == 1 and "Error:" in r.stderr
