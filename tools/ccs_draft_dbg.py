"""Debug: drafts of test_native_ccs_batch_matches_python_driver's chunks from the engine's POA alone (before and
after a native ccs batch), from the native ccs batch, and from the oracle's SparsePoa (first differing column)."""
import sys

import numpy as np

sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import pbccs_amd  # noqa: E402
from pbccs_amd import driver  # noqa: E402
from oracle import oracle  # noqa: E402
from test_poa_gpu import _synthetic_subreads  # noqa: E402


def chunks_of_test():
    rng = np.random.default_rng(8)
    chunks = []
    for reads in _synthetic_subreads(6, (300, 900), (3, 9), seed=55):
        chunks.append({"snr": [10.0, 7.0, 5.0, 11.0],
                       "reads": [{"seq": s, "flags": int(rng.choice([3, 3, 3, 1, 2]))} for s in reads]})
    chunks.append({"snr": [9.0, 9.0, 9.0, 9.0], "reads": [{"seq": "ACGTA"}]})
    chunks[0]["reads"].insert(0, {"seq": ""})
    chunks[1]["reads"].insert(2, {"seq": "", "flags": 3})
    return chunks


def first_diff(a, b):
    for i, (x, y) in enumerate(zip(a, b)):
        if x != y:
            return i
    return -1 if len(a) == len(b) else min(len(a), len(b))


def main():
    eng = pbccs_amd.Engine(0)
    chunks = chunks_of_test()
    bad = 0
    for cov in (None, 3, None, 3):
        orc = []
        for c in chunks:
            order = driver.filter_reads(c["reads"], 10)
            rs = [r["seq"] if r is not None else None for r in order]
            orc.append(oracle.sparse_poa(rs, None, cov)["consensus"] if rs else "")
        alone0 = [z["draft"] if z else None for st, z in driver.zmw_inputs_batch(chunks, max_poa_coverage=cov, engine=eng)]
        if len(sys.argv) > 1 and sys.argv[1] == "polish":   # the Arrow polish alone between the two POA runs
            ins = driver.zmw_inputs_batch(chunks, max_poa_coverage=cov, engine=eng)
            pbccs_amd.polish_zmws([z for st, z in ins if st is None], engine=eng)
            native = [z["draft"] if z else None for st, z in ins]
        else:
            native = [g["draft"] for g in driver.ccs_batch(chunks, engine=eng, max_poa_coverage=cov)]
        alone1 = [z["draft"] if z else None for st, z in driver.zmw_inputs_batch(chunks, max_poa_coverage=cov, engine=eng)]
        for i in range(len(chunks)):
            bad += int(not ((alone0[i] or "") == (native[i] or "") == (alone1[i] or "")))
            print(f"cov={cov} chunk={i} oracle_len={len(orc[i])} "
                  f"alone0={first_diff(alone0[i] or '', orc[i])} native={first_diff(native[i] or '', orc[i])} "
                  f"alone1={first_diff(alone1[i] or '', orc[i])}", flush=True)
    print("DISAGREE", bad, flush=True)


if __name__ == "__main__":
    main()
