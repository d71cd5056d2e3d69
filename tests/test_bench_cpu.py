"""CPU checks of bench.py's bookkeeping (no GPU): the algorithmic byte counts the roofline divides by
(config 3 forward 29.96 MB, backward 46.75 MB per frame), the frame partition of the N-rank path,
and the CPU-baseline host description."""
import bench


def test_alg_bytes_match_survey_8d():
    B, H, W, C, F = 1, 1024, 1024, 3, 50000
    V = 3 * F
    k, fwd, bwd = bench.alg_bytes(B, H, W, C, V, F)
    # fwd = 16V + 12F + 4CV + 4CHW (bg) + 4CHW (pixels); bwd adds grad outputs 16V + 4CV + 4CHW
    assert fwd == 16 * V + 12 * F + 4 * C * V + 2 * 4 * C * H * W
    assert bwd == 16 * V + 12 * F + 4 * C * V + 2 * 4 * C * H * W + 16 * V + 4 * C * V + 4 * C * H * W
    assert abs(fwd / 1e6 - 29.96) < 0.01 and abs(bwd / 1e6 - 46.75) < 0.01  # (SURVEY quotes 2 decimals)
    # per kernel: the roofline's backward kernel carries exactly SURVEY 8d's backward bytes (no
    # g-buffer, the colour input included); the forward's two launches split 8d's forward bytes
    assert k["grad_kernel"] == bwd
    assert k["setup_kernel"] == 12 * F + 16 * V
    assert k["raster_kernel"] == 2 * 4 * C * H * W + 4 * C * V
    assert k["setup_kernel"] + k["raster_kernel"] == fwd
    # batches scale linearly
    k2, fwd2, bwd2 = bench.alg_bytes(8, H, W, C, V, F)
    assert (fwd2, bwd2) == (8 * fwd, 8 * bwd) and all(k2[n] == 8 * k[n] for n in k)


def test_configs_and_host_info():
    assert bench.CONFIGS["c3"] == (1, 1024, 1024, 3, 50000, 16.0)
    assert bench.CONFIGS["c5"][0] == 8  # 64 frames over 8 GPUs: 8 per rank
    info = bench.host_cpu_info()
    assert set(info) == {"cpu_model", "nproc_online", "affinity_cpus"} and info["affinity_cpus"] >= 1
    assert bench.cpu_threads() >= 1


def test_cpu_share_evidence():
    """The CPU baseline records where its thread count comes from (SURVEY 8d asks for all host cores; the pool
    grants one GPU's job a share, OMP_NUM_THREADS on the box): cgroup quota / cpuset when readable."""
    share = bench.cpu_share()
    assert "OMP_NUM_THREADS" in share and share["nproc_online"] >= 1
    if "cgroup_cpu_max" in share and share["cgroup_cpu_max"].split()[0] != "max":
        assert share["cgroup_cpu_quota_cpus"] > 0
