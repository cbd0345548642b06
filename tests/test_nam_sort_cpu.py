"""CPU: the host's NAM ordering (load_sorted_nams, csrc/host/aln.cpp) equals
libstdc++'s std::sort by score -- the order the reference sorts a read's NAMs in
before shuffle_top_nams (src/aln.cpp:1962-1964) -- on 200 k random lists with ties."""
import os
import subprocess

from helpers import ROOT


def test_load_sorted_nams_is_std_sort(tmp_path):
    exe = tmp_path / "nam_sort_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", "-I", os.path.join(ROOT, "rabbitsalign_amd", "csrc", "host"),
                    os.path.join(ROOT, "tests", "cpp", "nam_sort_check.cpp"),
                    os.path.join(ROOT, "rabbitsalign_amd", "lib", "librsa_host.a"), "-lz", "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
