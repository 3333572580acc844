"""Multi-GPU host readiness: a rank's host threads follow
its share of the cgroup CPU quota. host/host_cpus.c sizes one persistent
thread pool per device (so per rank) from quota / LOCAL_WORLD_SIZE (and the
pinned CPUs): budget - 1 pool threads, and every engine of the rank runs
the per-frame items of its host phases on that pool plus its own calling
thread. So 8 ranks x 6 engines keep about one busy thread per quota CPU: at
most budget - 1 pool threads ever run items, beside the engines' callers.
The quota is faked with WEBP_AMD_CPU_QUOTA; the probe links host_cpus.c
alone (no GPU)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROBE = os.path.join(ROOT, "build", "hostpool", "pool_probe")


@pytest.fixture(scope="module")
def probe():
    os.makedirs(os.path.dirname(PROBE), exist_ok=True)
    subprocess.check_call(
        ["gcc", "-O1", "-std=gnu11", "-D__HIP_PLATFORM_AMD__",
         "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(ROOT, "libwebp_amd", "csrc"),
         "-I/opt/rocm/include", "-o", PROBE,
         os.path.join(ROOT, "tests", "hostpool", "pool_probe.c"),
         os.path.join(ROOT, "libwebp_amd", "csrc", "host", "host_cpus.c"),
         "-L/opt/rocm/lib", "-Wl,-rpath,/opt/rocm/lib", "-lamdhip64", "-lpthread"])
    return PROBE


def run(probe, quota, ranks, engines=6, items=64, width=15):
    env = dict(os.environ, WEBP_AMD_CPU_QUOTA=str(quota), LOCAL_WORLD_SIZE=str(ranks),
               LOCAL_RANK="0", WEBP_AMD_NO_PIN="1", HIP_VISIBLE_DEVICES="")
    env.pop("WEBP_AMD_THREADS", None)
    out = subprocess.run([probe, str(engines), str(items), str(width)], env=env,
                         capture_output=True, text=True, timeout=300, check=True).stdout.split()
    budget, threads, peak, done = int(out[1]), int(out[3]), int(out[5]), int(out[7])
    assert done == engines * items * 100          # every item ran, exactly once (probe checks)
    return budget, threads, peak


def test_quota_split_over_eight_ranks(probe):
    # a 16-CPU quota shared by 8 ranks: 2 threads per rank -> 1 pool thread
    budget, threads, peak = run(probe, 16, 8)
    assert budget == 2
    assert threads <= 6 + budget - 1          # the six engines' callers + the pool
    assert peak <= 6 + budget - 1


def test_pool_is_shared_by_the_engines(probe):
    online = os.cpu_count()
    budget, threads, peak = run(probe, 4 * online, 1, engines=3)
    assert budget == online                    # the quota exceeds the CPUs: the CPUs bind
    assert threads <= 3 + budget - 1 and peak <= 3 + budget - 1


def test_one_engine_gets_the_whole_pool(probe):
    budget, threads, peak = run(probe, 4, 1, engines=1, items=256)
    assert budget == 4
    assert peak == budget and threads == budget   # caller + 3 pool threads, all busy


def test_width_limits_a_job(probe):
    budget, threads, peak = run(probe, 8, 1, engines=1, items=256, width=1)
    assert peak <= 2                            # the caller + one pool thread


def test_node_quota_eight_ranks_six_engines(probe):
    # 8 ranks x 6 engines on a node quota of 8 x 3 CPUs: 2 pool threads a rank
    budget, threads, peak = run(probe, 24, 8, engines=6)
    assert budget == 3 and peak <= 6 + 2
