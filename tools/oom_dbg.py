"""Debug: tests/test_schedule.py's out-of-memory rerun test with most of the device's memory held by another
allocation (as earlier tests' engines hold it in a full GPU run), so the fills cannot take in-kernel growth
headroom.  Usage: python tools/oom_dbg.py [GB to leave free] [part: all | queue]"""
import os
import sys

sys.path.insert(0, os.getcwd())
sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import torch  # noqa: E402


class _MP:
    def setenv(self, k, v):
        os.environ[k] = v


def main():
    leave = float(sys.argv[1]) if len(sys.argv) > 1 else 20.0
    part = sys.argv[2] if len(sys.argv) > 2 else "all"
    free, total = torch.cuda.mem_get_info(0)
    hold = max(0, int(free - leave * (1 << 30)))
    blocks = []
    while hold > 0:   # in 16 GB pieces
        n = min(hold, 16 << 30)
        blocks.append(torch.empty(n, dtype=torch.uint8, device="cuda:0"))
        hold -= n
    print(f"held {sum(b.numel() for b in blocks) / 2**30:.1f} GB of {free / 2**30:.1f} GB free", flush=True)
    if part == "all":
        import test_schedule
        test_schedule.test_out_of_memory_batches_are_rerun_with_identical_results(_MP())
        print("passed", flush=True)
        return
    import pbccs_amd
    from pbccs_amd import synth
    zs = synth.make_zmws(24, 2000, 10, seed=31)
    small = synth.make_zmws(2, 600, 6, seed=32)
    ref = pbccs_amd.polish_zmws(zs + small, engine=pbccs_amd.Engine(0))
    if os.environ.get("OOM_DBG_NO_CAP") != "1":   # OOM_DBG_NO_CAP=1: no capped pool, so no batch runs out of memory
        os.environ["PBCCS_POOL_CAP_MB"] = "200"
    eng = pbccs_amd.Engine(0)
    eng.set_concurrency(2)
    got = pbccs_amd.polish_stream(zs + small, pbccs_amd.ConsensusSettings(zmws_per_batch=24), eng)
    print("oom_retries", eng.counters()["oom_retries"], flush=True)
    bad = 0
    for i, (a, b) in enumerate(zip(got, ref)):
        keys = [k for k in ("status", "n_tested", "n_applied", "consensus", "add_read_results") if a[k] != b[k]]
        if keys:
            bad += 1
            print(i, keys, {k: (a[k], b[k]) for k in ("status", "n_tested", "n_applied")}, flush=True)
    print("differing ZMWs", bad, flush=True)


if __name__ == "__main__":
    main()
