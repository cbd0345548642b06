"""CPU: the host pipeline is deterministic and the C restatement engine equals the
reference's own hot-path code (randstrobes/nam/ssw.c) end to end."""
import os

import pytest

from e2e import CPU_PORT, CPU_REF, make_dataset, map_reads, sam_body


@pytest.fixture(scope="module")
def data(tmp_path_factory):
    d = tmp_path_factory.mktemp("e2e_cpu")
    return d, make_dataset(str(d), pairs=3000, ref_len=200_000, cpu_index=True)


@pytest.mark.skipif(not os.path.exists(CPU_REF), reason="reference build absent")
def test_port_equals_reference_hot_path(data):
    d, (fa, reads) = data
    map_reads(CPU_PORT, fa, reads, str(d / "port.sam"), "-t", "2", "--chunk-size", "700")
    map_reads(CPU_REF, fa, reads, str(d / "ref.sam"), "-t", "2", "--chunk-size", "700")
    assert sam_body(d / "port.sam") == sam_body(d / "ref.sam")


@pytest.mark.parametrize("chunk", ["100", "500"])
def test_thread_and_chunk_invariance(data, chunk):
    # the insert-size estimate freezes inside some chunk's part(); the parallel stage
    # opens right there (early freeze), and the output must not depend on it
    d, (fa, reads) = data
    map_reads(CPU_PORT, fa, reads, str(d / "t1.sam"), "-t", "1", "--chunk-size", chunk)
    for t in ("4", "8"):
        map_reads(CPU_PORT, fa, reads, str(d / f"t{t}.sam"), "-t", t, "--chunk-size", chunk)
        assert sam_body(d / "t1.sam") == sam_body(d / f"t{t}.sam")


@pytest.mark.parametrize("se", [True, False])
def test_engine_error_is_reported_not_aborted(tmp_path, se):
    """An engine call that throws (a failed GPU call in the product engine) ends the
    run with an error message and exit status 1, on the single-end path as on the
    paired-end one -- never std::terminate (SE worker had no handler)."""
    import subprocess
    fa, reads = make_dataset(str(tmp_path), pairs=2000, ref_len=100_000, cpu_index=True, se=se)
    env = dict(os.environ, RSA_TEST_FAIL_EXTEND="2")
    r = subprocess.run([CPU_PORT, "--use-index", "-t", "4", "--chunk-size", "200", "-o", str(tmp_path / "x.sam"),
                        fa, *reads], capture_output=True, text=True, env=env)
    assert r.returncode == 1, (r.returncode, r.stderr[-500:])
    assert "injected extend failure" in r.stderr


@pytest.mark.parametrize("threads", ["1", "7"])
def test_thread_count_invariance(data, threads):
    """The SAM does not depend on the number of host workers (the single-worker
    timeline until the insert-size estimate freezes, chunk-index seeding after)."""
    d, (fa, reads) = data
    base = str(d / "t4.sam")
    map_reads(CPU_PORT, fa, reads, base, "-t", "4", "--chunk-size", "200")
    out = str(d / f"t{threads}.sam")
    map_reads(CPU_PORT, fa, reads, out, "-t", threads, "--chunk-size", "200")
    assert sam_body(base) == sam_body(out)


def test_shared_substring_on_engine_equals_host(tmp_path):
    """rescue_mate_part's has_shared_substring: once the insert-size estimate is frozen
    the engine makes the test with the rescue SW job (SwJob::shared_k; the device kernel in
    the GPU engine, the host function in these CPU engines) and store_rescue writes the
    unaligned result.  A third of the second mates are replaced by random sequence, so
    their rescues find no shared substring; the SAM must equal the all-host test's
    (RSA_SHARED_ON_ENGINE=0), for both CPU engines."""
    import random
    fa, reads = make_dataset(str(tmp_path), pairs=3000, ref_len=200_000, cpu_index=True)
    rnd = random.Random(5)
    with open(reads[1]) as f:
        lines = f.read().split("\n")
    for r in range(0, len(lines) - 3, 4):
        if (r // 4) % 3 == 1:
            lines[r + 1] = "".join(rnd.choice("ACGT") for _ in lines[r + 1])
    with open(reads[1], "w") as f:
        f.write("\n".join(lines))
    outs = {}
    for binary in (CPU_PORT, CPU_REF):
        if not os.path.exists(binary):
            continue
        for on in ("1", "0"):
            out = str(tmp_path / f"{os.path.basename(binary)}_{on}.sam")
            old = os.environ.get("RSA_SHARED_ON_ENGINE")
            os.environ["RSA_SHARED_ON_ENGINE"] = on
            try:
                map_reads(binary, fa, reads, out, "-t", "4", "--chunk-size", "300")
            finally:
                if old is None:
                    del os.environ["RSA_SHARED_ON_ENGINE"]
                else:
                    os.environ["RSA_SHARED_ON_ENGINE"] = old
            outs[(binary, on)] = sam_body(out)
        assert outs[(binary, "1")] == outs[(binary, "0")], binary
    assert len(outs) >= 2
