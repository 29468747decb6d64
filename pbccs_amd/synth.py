"""Deterministic synthetic ZMWs for the benchmark configs (BASELINE.md "Inputs").

Per ZMW: truth = iid ACGT of length J; draft (POA stand-in) = truth with 0.5% insertions, 0.5% deletions,
0.2% substitutions; subreads = truth with 7% insertions (geometric, before each base), 4% deletions, 1%
substitutions, odd passes reverse-complemented (REVERSE strand), each mapped over the whole draft.
There is no BAM input in the reference tree (tests/data holds one FASTA ZMW), so configs #2-#5 use this.
"""
import numpy as np

BASES = np.frombuffer(b"ACGT", dtype=np.uint8)
COMP = np.zeros(256, dtype=np.uint8)
for a, b in zip(b"ACGT", b"TGCA"):
    COMP[a] = b


def _mutate(rng, seq, p_ins, p_del, p_sub):
    n = seq.shape[0]
    keep = rng.random(n) >= p_del
    sub = rng.random(n) < p_sub
    out = seq.copy()
    if sub.any():
        # a different base: shift by 1..3 in base-index space
        idx = np.searchsorted(BASES, out[sub])
        out[sub] = BASES[(idx + rng.integers(1, 4, size=int(sub.sum()))) % 4]
    ins_counts = rng.geometric(1.0 - p_ins, size=n) - 1 if p_ins > 0 else np.zeros(n, dtype=np.int64)
    total_ins = int(ins_counts.sum())
    ins_bases = BASES[rng.integers(0, 4, size=total_ins)]
    kept = keep.astype(np.int64)
    lens = ins_counts + kept
    res = np.empty(int(lens.sum()), dtype=np.uint8)
    ends = np.cumsum(lens)
    starts = ends - lens
    # insertions first (before the base), then the kept base
    pos_ins = np.repeat(starts, ins_counts) + (np.arange(total_ins) - np.repeat(np.cumsum(ins_counts) - ins_counts, ins_counts))
    res[pos_ins] = ins_bases
    res[ends[keep] - 1] = out[keep]
    return res


def make_zmw(rng, length, passes, snr=(10.0, 7.0, 5.0, 11.0), read_errors=(0.07, 0.04, 0.01)):
    truth = BASES[rng.integers(0, 4, size=length)]
    draft = _mutate(rng, truth, 0.005, 0.005, 0.002)
    reads = []
    for k in range(passes):
        r = _mutate(rng, truth, *read_errors)
        strand = k % 2
        if strand == 1:
            r = COMP[r[::-1]]
        reads.append({"seq": r.tobytes().decode(), "strand": strand, "ts": 0, "te": int(draft.shape[0])})
    return {"truth": truth.tobytes().decode(), "draft": draft.tobytes().decode(), "snr": list(snr), "reads": reads}


def make_zmws(n, length, passes, seed, snr=(10.0, 7.0, 5.0, 11.0), length_range=None, passes_range=None,
              random_snr=False):
    """n ZMWs.  length_range/passes_range (inclusive) draw per-ZMW sizes (config #4)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    out = []
    for _ in range(n):
        L = int(rng.integers(length_range[0], length_range[1] + 1)) if length_range else length
        P = int(rng.integers(passes_range[0], passes_range[1] + 1)) if passes_range else passes
        s = tuple(float(x) for x in rng.uniform(4.0, 20.0, size=4)) if random_snr else snr
        out.append(make_zmw(rng, L, P, s))
    return out


def make_smrtcell(n, seed=4):
    """configs[4]: a SMRT cell's mix of the configs #2-#4 shapes, one third each, the
    shape of every ZMW drawn from the seeded stream (so any prefix of the cell is the same mix)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    out = []
    for _ in range(n):
        kind = int(rng.integers(0, 3))
        if kind == 0:
            z = make_zmw(rng, 2000, 10)
        elif kind == 1:
            z = make_zmw(rng, 10000, 8)
        else:
            L = int(rng.integers(500, 20001))
            P = int(rng.integers(3, 31))
            z = make_zmw(rng, L, P, tuple(float(x) for x in rng.uniform(4.0, 20.0, size=4)))
        z["kind"] = ("2kb", "10kb", "mixed")[kind]
        out.append(z)
    return out


class SmrtCell:
    """configs[4] generated lazily: ZMW i of the cell is drawn from its own seeded stream (seed, i), so any rank
    can materialise any chunk of the cell without generating the rest (150k ZMWs of strings per rank would be
    ~14 GB of Python objects).  Shape (kind, insert length, passes, SNR) and sequences come from two separate
    streams, so the work queue can order the whole cell by cost from the shapes alone.  One third each of the
    configs #2-#4 shapes, as make_smrtcell.  Indexing returns make_zmw's dict plus "kind"."""
    KINDS = ("2kb", "10kb", "mixed")

    def __init__(self, n, seed=4):
        self.n = int(n)
        self.seed = int(seed)
        self._shapes = None

    def __len__(self):
        return self.n

    def shape(self, i):
        if self._shapes is not None:
            return self._shapes[i]
        rng = np.random.Generator(np.random.PCG64(np.random.SeedSequence([self.seed, int(i), 0])))
        kind = int(rng.integers(0, 3))
        if kind == 0:
            return kind, 2000, 10, (10.0, 7.0, 5.0, 11.0)
        if kind == 1:
            return kind, 10000, 8, (10.0, 7.0, 5.0, 11.0)
        L = int(rng.integers(500, 20001))
        P = int(rng.integers(3, 31))
        return kind, L, P, tuple(float(x) for x in rng.uniform(4.0, 20.0, size=4))

    def shapes(self):
        if self._shapes is None:
            self._shapes = [self.shape(i) for i in range(self.n)]
        return self._shapes

    def costs(self):
        """shard.zmw_cost's estimate (draft length x read bases) from the shapes: L x (1.03 L) x passes."""
        return [max(1, L) * max(1, int(1.03 * L) * P) for _, L, P, _ in self.shapes()]

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[k] for k in range(*i.indices(self.n))]
        if not 0 <= i < self.n:
            raise IndexError(i)
        kind, L, P, snr = self.shape(i)
        rng = np.random.Generator(np.random.PCG64(np.random.SeedSequence([self.seed, int(i), 1])))
        z = make_zmw(rng, L, P, snr)
        z["kind"] = self.KINDS[kind]
        return z

    def __iter__(self):
        return (self[i] for i in range(self.n))


CONFIGS = {
    # name: (n_zmws, insert length, passes, seed) -- BASELINE.json configs[1..3]
    "2kb_10pass": dict(length=2000, passes=10, seed=1),
    "10kb_8pass": dict(length=10000, passes=8, seed=2),
    "mixed": dict(length=None, passes=None, seed=3, length_range=(500, 20000), passes_range=(3, 30), random_snr=True),
}


# Quiver model parameters of the synthetic Quiver workload (a QvModelParams set of the reference's magnitude;
# the same set tests/test_quiver_gpu.py scores with)
QUIVER_PARAMS = dict(Match=-0.2, Mismatch=-8.0, MismatchS=-0.15, Branch=-3.5, BranchS=-0.12, DeletionN=-7.5,
                     DeletionWithTag=-4.5, DeletionWithTagS=-0.2, Nce=-6.0, NceS=-0.1, Merge=[-3.0, -3.2, -2.9, -3.1],
                     MergeS=[-0.1, -0.12, -0.09, -0.11])

QUIVER_READ_ERRORS = (0.04, 0.03, 0.01)
QUIVER_SCORE_DIFF = 18.0   # at 12.5 the FP32 band loses nearly every 2 kb read to an alpha/beta mismatch


def make_quiver_zmws(n, length, passes, seed, read_errors=QUIVER_READ_ERRORS):
    """n Quiver ZMWs: make_zmw's draft and mapped reads (at read_errors ins/del/sub rates, a little
    cleaner than configs[1]'s; scored at QUIVER_SCORE_DIFF), each read with five QV feature tracks as numpy arrays (InsQv, SubsQv, DelQv, MergeQv: float32
    uniform integers in [0, 25); DelTag: uint8 character codes uniform over ACGTN)."""
    zrng = np.random.Generator(np.random.PCG64(seed))
    rng = np.random.Generator(np.random.PCG64(seed + 17))
    out = []
    for z in [make_zmw(zrng, length, passes, read_errors=read_errors) for _ in range(n)]:
        reads = []
        for r in z["reads"]:
            m = len(r["seq"])
            f = {"ins": rng.integers(0, 25, m).astype(np.float32), "subs": rng.integers(0, 25, m).astype(np.float32),
                 "del": rng.integers(0, 25, m).astype(np.float32),
                 "del_tag": np.frombuffer(b"ACGTN", dtype=np.uint8)[rng.integers(0, 5, m)].copy(),
                 "merge": rng.integers(0, 25, m).astype(np.float32)}
            reads.append(dict(r, features=f))
        out.append({"tpl": z["draft"], "reads": reads})
    return out
