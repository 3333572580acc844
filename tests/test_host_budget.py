"""Multi-GPU host readiness: a rank's host threads follow
its share of the cgroup CPU quota. host/host_cpus.c sizes one pool per
process from quota / LOCAL_WORLD_SIZE (and the pinned CPUs), and every
engine draws the helper threads of its host phases from it, so 8 ranks x 6
engines stay at about one busy thread per quota CPU: the helpers in flight
never exceed the budget minus one, whatever the number of engines (each
engine's calling thread works its own phase and is the only thread beyond
the budget). The quota is faked
with WEBP_AMD_CPU_QUOTA; the probe links host_cpus.c alone (no GPU)."""
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


def run(probe, quota, ranks, engines=6, want=15):
    env = dict(os.environ, WEBP_AMD_CPU_QUOTA=str(quota), LOCAL_WORLD_SIZE=str(ranks),
               LOCAL_RANK="0", WEBP_AMD_NO_PIN="1", HIP_VISIBLE_DEVICES="")
    env.pop("WEBP_AMD_THREADS", None)
    out = subprocess.run([probe, str(engines), str(want)], env=env, capture_output=True,
                         text=True, timeout=120, check=True).stdout.split()
    return int(out[1]), int(out[3]), int(out[5])


def test_quota_split_over_eight_ranks(probe):
    # a 16-CPU quota shared by 8 ranks: 2 threads per rank
    budget, peak, helpers = run(probe, 16, 8)
    assert budget == 2
    assert helpers <= budget - 1
    assert peak <= 6 + budget - 1       # six callers + the pool's helpers


def test_pool_caps_helpers_across_engines(probe):
    online = os.cpu_count()
    budget, peak, helpers = run(probe, 4 * online, 1, engines=3, want=15)
    assert budget == online             # the quota exceeds the CPUs: the CPUs bind
    assert helpers <= budget - 1
    assert peak <= budget + 2


def test_node_quota_one_thread_per_cpu(probe):
    # 8 ranks x 6 engines on a node quota of 8 x 3 CPUs
    budget, peak, helpers = run(probe, 24, 8, engines=6)
    assert budget == 3 and helpers <= 2 and peak <= 8
    # one engine alone gets the whole pool
    budget, peak, helpers = run(probe, 24, 8, engines=1)
    assert helpers == budget - 1 and peak == budget
