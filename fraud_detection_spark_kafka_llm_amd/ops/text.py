"""Text featurization ops: packed UTF-8 columns, string tables and the fused featurize+score op.

``featurize_score`` runs the whole Tokenizer -> StopWordsRemover -> HashingTF|CountVectorizerModel
(-> IDFModel) (-> LogisticRegressionModel | tree ensemble) chain of a Spark pipeline in ONE
native launch (``csrc/text_kernels.hip`` on gfx950, ``csrc/text_cpu.cpp`` on the host). The rare
documents the GPU kernel cannot hold in LDS (longer than 4 KiB, > 1024 kept tokens) or that need
full Unicode lowercasing are finished by the host path and patched into the device outputs.

Reference semantics: SURVEY.md Appendix A.1-A.5; /root/reference/fraud_detection_spark.py:47-54
(feature stages) and the shipped dialogue_classification_model stages 0-4.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Optional, Sequence

import numpy as np
import torch

from . import native
from .oracle import murmur3_x86_32

# keep in sync with csrc/common.h
FLAG_CLEAN = 1 << 0
FLAG_BINARY = 1 << 1
FLAG_WRITE_CSR = 1 << 2
FLAG_IDF = 1 << 3
FLAG_LR = 1 << 4
FLAG_TREES = 1 << 5
FLAG_VOCAB = 1 << 6
FLAG_STOPWORDS = 1 << 7
FLAG_CMP_LESS = 1 << 8
FLAG_PRELOWERED = 1 << 9
STATUS_OK, STATUS_TOO_LONG, STATUS_NEEDS_HOST = 0, 1, 2
PAD = 16


# ----------------------------------------------------------------------------- packed text
class PackedText:
    """A string column as one UTF-8 byte buffer + int64 offsets (``offsets[i]..offsets[i+1]``).

    The byte buffer is zero-padded by ``PAD`` bytes so the GPU kernel's dword loads never run
    past the allocation.
    """

    __slots__ = ("data", "offsets", "_strings")

    def __init__(self, data: torch.Tensor, offsets: torch.Tensor, strings: Optional[list] = None):
        self.data = data
        self.offsets = offsets
        self._strings = strings

    @classmethod
    def from_strings(cls, texts: Sequence[Optional[str]], pin: bool = False) -> "PackedText":
        enc = [(t if t is not None else "").encode("utf-8") for t in texts]
        lens = np.fromiter((len(b) for b in enc), dtype=np.int64, count=len(enc))
        offs = np.zeros(len(enc) + 1, dtype=np.int64)
        np.cumsum(lens, out=offs[1:])
        buf = np.zeros(int(offs[-1]) + PAD, dtype=np.uint8)
        if enc:
            joined = b"".join(enc)
            buf[: len(joined)] = np.frombuffer(joined, dtype=np.uint8)
        data = torch.from_numpy(buf)
        off = torch.from_numpy(offs)
        if pin and torch.cuda.is_available():
            data, off = data.pin_memory(), off.pin_memory()
        return cls(data, off, list(texts))

    @classmethod
    def from_bytes(cls, data: np.ndarray, offsets: np.ndarray) -> "PackedText":
        n = int(offsets[-1])
        buf = np.zeros(n + PAD, dtype=np.uint8)
        buf[:n] = data[:n]
        return cls(torch.from_numpy(buf), torch.from_numpy(np.ascontiguousarray(offsets, dtype=np.int64)))

    def __len__(self) -> int:
        return int(self.offsets.numel()) - 1

    @property
    def device(self) -> torch.device:
        return self.data.device

    @property
    def nbytes(self) -> int:
        return int(self.offsets[-1])

    def to(self, device, non_blocking: bool = False) -> "PackedText":
        device = torch.device(device)
        if self.data.device == device:
            return self
        return PackedText(self.data.to(device, non_blocking=non_blocking),
                          self.offsets.to(device, non_blocking=non_blocking), self._strings)

    def strings(self) -> list:
        if self._strings is None:
            d = self.data.cpu().numpy()
            o = self.offsets.cpu().numpy()
            self._strings = [bytes(d[o[i]:o[i + 1]]).decode("utf-8", errors="replace") for i in range(len(self))]
        return self._strings

    def take(self, ids: Sequence[int]) -> "PackedText":
        s = self.strings()
        return PackedText.from_strings([s[i] for i in ids])


# ----------------------------------------------------------------------------- string tables
class StrTable:
    """Open-addressing table of UTF-8 strings keyed by murmur3(seed 42) (load factor <= 0.5).

    Mirrors ``fdx::StrTable``: ``slots`` (entry index or -1), ``hashes``, ``offs``, ``bytes``.
    Entry ``i`` is ``words[i]``; lookups verify bytes so collisions cannot change results.
    """

    def __init__(self, words: Sequence[str]):
        self.words = list(words)
        enc = [w.encode("utf-8") for w in self.words]
        n = len(enc)
        size = 16
        while size < 2 * max(n, 1):
            size <<= 1
        hashes = np.array([murmur3_x86_32(b, 42) for b in enc], dtype=np.uint32)
        slots = np.full(size, -1, dtype=np.int32)
        mask = size - 1
        seen = set()
        for i, (b, h) in enumerate(zip(enc, hashes)):
            if b in seen:
                continue
            seen.add(b)
            j = int(h) & mask
            while slots[j] >= 0:
                j = (j + 1) & mask
            slots[j] = i
        offs = np.zeros(n + 1, dtype=np.int64)
        np.cumsum([len(b) for b in enc], out=offs[1:])
        self._host = (torch.from_numpy(slots), torch.from_numpy(hashes.view(np.int32).copy()),
                      torch.from_numpy(offs),
                      torch.from_numpy(np.frombuffer(b"".join(enc) + b"\0", dtype=np.uint8).copy()))
        self._dev: dict = {}

    def tensors(self, device) -> list:
        device = torch.device(device)
        if device.type == "cpu":
            return list(self._host)
        key = str(device)
        if key not in self._dev:
            self._dev[key] = [t.to(device) for t in self._host]
        return self._dev[key]


# ----------------------------------------------------------------------------- specs / scorers
@dataclass
class FeatureSpec:
    """The fused text prefix of a pipeline (Tokenizer -> StopWordsRemover -> TF)."""
    clean: bool = True                       # regexp_replace(lower(x), "[^a-zA-Z ]", "") first
    stopwords: Optional[Sequence[str]] = None
    num_features: int = 1 << 18              # HashingTF.numFeatures (Spark default 262144)
    binary: bool = False
    vocab: Optional[Sequence[str]] = None    # CountVectorizerModel vocabulary (replaces hashing)
    min_tf: float = 1.0
    _tables: dict = field(default_factory=dict, repr=False, compare=False)

    @property
    def dim(self) -> int:
        return len(self.vocab) if self.vocab is not None else int(self.num_features)

    def stop_table(self) -> Optional[StrTable]:
        if not self.stopwords:
            return None
        if "stop" not in self._tables:
            self._tables["stop"] = StrTable([w.lower() for w in self.stopwords])
        return self._tables["stop"]

    def vocab_table(self) -> Optional[StrTable]:
        if self.vocab is None:
            return None
        if "vocab" not in self._tables:
            self._tables["vocab"] = StrTable(self.vocab)
        return self._tables["vocab"]


class _DeviceCached:
    def _cached(self, device, build):
        device = torch.device(device)
        cache = self.__dict__.setdefault("_devcache", {})
        key = str(device)
        if key not in cache:
            cache[key] = build(device)
        return cache[key]


class LinearScorer(_DeviceCached):
    """Binary logistic-regression margin ``w . x + b`` (fp64)."""

    def __init__(self, w: np.ndarray, b: float):
        self.w = np.asarray(w, dtype=np.float64)
        self.b = float(b)

    def weights(self, device) -> torch.Tensor:
        return self._cached(device, lambda d: torch.from_numpy(self.w).to(d))


class TreeArrays(_DeviceCached):
    """Flattened ensemble (see ``fdx::TreeEnsemble``). ``K`` leaf values per node."""

    def __init__(self, feat, thr, left, right, leaf, roots, weights, K: int, cmp_less: bool):
        self.feat = np.ascontiguousarray(feat, dtype=np.int32)
        self.thr = np.ascontiguousarray(thr, dtype=np.float64)
        self.left = np.ascontiguousarray(left, dtype=np.int32)
        self.right = np.ascontiguousarray(right, dtype=np.int32)
        self.leaf = np.ascontiguousarray(leaf, dtype=np.float64).reshape(-1)
        self.roots = np.ascontiguousarray(roots, dtype=np.int32)
        self.tree_weights = np.ascontiguousarray(weights, dtype=np.float64)
        self.K = int(K)
        self.cmp_less = bool(cmp_less)
        n = self.feat.size
        if not (self.thr.size == self.left.size == self.right.size == n and self.leaf.size == n * self.K):
            raise ValueError("inconsistent tree arrays")
        internal = self.feat >= 0
        for arr in (self.left, self.right):
            if np.any(internal & ((arr < 0) | (arr >= n))):
                raise ValueError("child index out of range")
        if np.any((self.roots < 0) | (self.roots >= max(n, 1))):
            raise ValueError("root index out of range")

    @property
    def num_trees(self) -> int:
        return int(self.roots.size)

    def tensors(self, device) -> list:
        return self._cached(device, lambda d: [torch.from_numpy(a).to(d) for a in (
            self.feat, self.thr, self.left, self.right, self.leaf, self.roots, self.tree_weights)])

    def max_feature(self) -> int:
        return int(self.feat.max()) if self.feat.size else -1


# ----------------------------------------------------------------------------- results
class FeatureResult:
    """Outputs of one fused launch. ``raw`` is ``[D, K]`` fp64 (LR: margin; trees: raw sums)."""

    def __init__(self, nnz, ntok, raw, status, idx, val, base, dim):
        self.nnz, self.ntok, self.raw, self.status = nnz, ntok, raw, status
        self.idx, self.val, self.base, self.dim = idx, val, base, dim

    def __len__(self) -> int:
        return int(self.nnz.numel())

    def csr(self):
        """Compacted CSR ``(indptr int64[D+1], indices int32[nnz], values float32[nnz])``."""
        if self.idx is None:
            raise ValueError("featurize_score ran without want_csr=True")
        nnz = self.nnz.to(torch.int64)
        D = nnz.numel()
        indptr = torch.zeros(D + 1, dtype=torch.int64, device=nnz.device)
        torch.cumsum(nnz, 0, out=indptr[1:])
        total = int(indptr[-1])
        return indptr, *self._compact(nnz, indptr, total)

    def _compact(self, nnz: torch.Tensor, indptr: torch.Tensor, total: int) -> tuple:
        """Gather every row's entries from its slot at ``base[r]`` into CSR order. The source
        position of each output entry is a running sum of steps: +1 inside a row, and at the
        first entry of each non-empty row the jump from the previous non-empty row's last entry
        to ``base[r]`` — one scatter over the rows plus one scan, where a per-entry row index
        (``repeat_interleave``: one thread per row writing its entries serially, ~6 ms per
        500K-row chunk on the MI355X, profiles/r3s4/bench_full_kernel_stats.csv) and two
        gathers through it were."""
        dev = nnz.device
        if total == 0:
            return self.idx[:0], self.val[:0]
        nz = torch.nonzero(nnz).flatten()
        base = self.base.to(torch.int64)[nz]
        starts = indptr[nz]
        step = torch.ones(total, dtype=torch.int64, device=dev)
        jump = base.clone()
        jump[1:] -= base[:-1] + nnz[nz[:-1]] - 1       # from the previous row's last entry
        step[starts] = jump
        pos = torch.cumsum(step, 0)
        return self.idx[pos], self.val[pos]


def _flags(spec: FeatureSpec, idf, lr, trees, want_csr: bool) -> int:
    f = 0
    if spec.clean:
        f |= FLAG_CLEAN
    if spec.binary:
        f |= FLAG_BINARY
    if want_csr:
        f |= FLAG_WRITE_CSR
    if idf is not None:
        f |= FLAG_IDF
    if lr is not None:
        f |= FLAG_LR
    if trees is not None:
        f |= FLAG_TREES
        if trees.cmp_less:
            f |= FLAG_CMP_LESS
    if spec.vocab is not None:
        f |= FLAG_VOCAB
    if spec.stopwords:
        f |= FLAG_STOPWORDS
    return f


def csr_capacity(nbytes: int, docs: int) -> int:
    """Entries of the fused featurizer's CSR scratch for ``docs`` documents of ``nbytes`` bytes
    (csrc/scoring.h csr_capacity: at most L / 2 + 2 distinct terms per L-byte document)."""
    return (int(nbytes) >> 1) + 2 * int(docs) + 1


def csr_slots(starts: torch.Tensor, index: torch.Tensor) -> torch.Tensor:
    """First scratch slot of each document (csrc/scoring.h csr_slot): start / 2 + 2 * index."""
    return (starts >> 1) + 2 * index


LONG_DOC_BYTES = 65536   # documents up to this size stay on the GPU (long-dialogue kernel)


def _launch(C, text: PackedText, spec, flags, idf_t, lr, trees, out, device, only=None, threads=0, long_docs=None):
    nnz, ntok, raw, status, idx, val = out
    st = spec.stop_table()
    vt = spec.vocab_table()
    K = trees.K if trees is not None else 1
    C.featurize_score(
        text.data, text.offsets, flags, spec.dim,
        st.tensors(device) if st else None, vt.tensors(device) if vt else None,
        float(spec.min_tf), idf_t, lr.weights(device) if lr is not None else None,
        float(lr.b) if lr is not None else 0.0,
        trees.tensors(device) if trees is not None else None, K,
        idx, val, nnz, ntok, raw, status, only, int(threads), long_docs)


def featurize_score(text: PackedText, spec: FeatureSpec, idf: Optional[torch.Tensor] = None,
                    lr: Optional[LinearScorer] = None, trees: Optional[TreeArrays] = None,
                    want_csr: bool = False, device=None, threads: int = 0,
                    fix_fallbacks: bool = True) -> FeatureResult:
    """Run the fused pipeline over ``text`` on ``device`` (default: where ``text`` lives)."""
    if lr is not None and trees is not None:
        raise ValueError("one scorer per launch")
    C = native.lib()
    device = torch.device(device) if device is not None else text.device
    host_text = text
    text = text.to(device, non_blocking=True)
    D = len(text)
    if trees is not None and trees.max_feature() >= spec.dim:
        raise ValueError("tree ensemble references a feature outside the feature space")
    idf_t = None
    if idf is not None:
        idf_t = idf.to(device=device, dtype=torch.float64)
        if idf_t.numel() < spec.dim:
            raise ValueError("idf vector shorter than the feature space")
    K = trees.K if trees is not None else 1
    cap = csr_capacity(text.data.numel(), D) if want_csr else 1
    i32 = dict(dtype=torch.int32, device=device)
    out = (torch.zeros(D, **i32), torch.zeros(D, **i32),
           torch.zeros((D, K), dtype=torch.float64, device=device), torch.full((D,), -1, **i32),
           torch.empty(cap, **i32), torch.empty(cap, dtype=torch.float32, device=device))
    flags = _flags(spec, idf_t, lr, trees, want_csr)
    _launch(C, text, spec, flags, idf_t, lr, trees, out, device, None, threads)
    nnz, ntok, raw, status, idx, val = out
    if device.type == "cuda" and D:
        # documents over the streaming kernel's LDS capacity: rerun them on the long-dialogue kernel
        lens = text.offsets[1:] - text.offsets[:-1]
        long_docs = torch.nonzero((status == STATUS_TOO_LONG) & (lens <= LONG_DOC_BYTES)).flatten()
        if long_docs.numel():
            _launch(C, text, spec, flags, idf_t, lr, trees, out, device, None, threads,
                    long_docs.to(torch.int32).contiguous())
    base = csr_slots(text.offsets[:-1], torch.arange(D, device=device, dtype=torch.int64))
    res = FeatureResult(nnz, ntok, raw, status, idx if want_csr else None, val if want_csr else None, base, spec.dim)
    if device.type == "cuda" and D:
        _long_docs_on_device(res, text, host_text, spec, idf_t, lr, trees, want_csr, device)
    if fix_fallbacks and D:
        bad = torch.nonzero(status != STATUS_OK).flatten()
        if bad.numel():
            _finish_on_host(res, host_text, bad.cpu().numpy(), spec, idf, lr, trees, want_csr, flags)
    return res


def _long_docs_on_device(res: FeatureResult, text: PackedText, host_text: PackedText, spec, idf_t, lr, trees,
                         want_csr: bool, device) -> None:
    """Dialogues over LONG_DOC_BYTES: segmented device path (ops/longdoc.py), patched into ``res``."""
    from .longdoc import featurize_long

    lens = text.offsets[1:] - text.offsets[:-1]
    very = torch.nonzero((res.status == STATUS_TOO_LONG) & (lens > LONG_DOC_BYTES)).flatten()
    if not very.numel():
        return
    docs = very.cpu().numpy()
    host_buf = host_text.data.cpu().numpy() if host_text.data.is_cuda else host_text.data.numpy()
    done, raw, nnz, ntok, csr = featurize_long(text.data, host_buf, text.offsets.cpu().numpy(), docs, spec, idf_t,
                                               lr, trees, device)
    if not done.any():
        return
    d = torch.from_numpy(docs[done].astype(np.int64)).to(device)
    res.raw[d] = raw if raw.shape[1] == res.raw.shape[1] else raw[:, : res.raw.shape[1]]
    res.nnz[d] = nnz.to(device)
    res.ntok[d] = ntok.to(device)
    res.status[d] = STATUS_OK
    if want_csr:
        indptr, col, v = csr
        per = indptr[1:] - indptr[:-1]
        total = int(indptr[-1])
        owner = torch.repeat_interleave(torch.arange(per.numel(), device=device), per, output_size=total)
        pos = res.base[d][owner] + (torch.arange(total, device=device) - indptr[owner])
        res.idx[pos] = col
        res.val[pos] = v.to(torch.float32)


def _finish_on_host(res: FeatureResult, text: PackedText, bad: np.ndarray, spec, idf, lr, trees,
                    want_csr: bool, flags: int) -> None:
    """Re-run flagged documents on the host path and patch them into ``res``."""
    strings = text.strings()
    sub_strings = []
    for i in bad:
        s = strings[int(i)] or ""
        if not spec.clean:
            s = s.lower()     # Java toLowerCase (default locale) ~ Python full case mapping
        sub_strings.append(s)
    sub = PackedText.from_strings(sub_strings)
    sub_flags = flags | (0 if spec.clean else FLAG_PRELOWERED)
    D = len(sub)
    K = trees.K if trees is not None else 1
    cap = csr_capacity(sub.data.numel(), D) if want_csr else 1
    i32 = dict(dtype=torch.int32)
    out = (torch.zeros(D, **i32), torch.zeros(D, **i32), torch.zeros((D, K), dtype=torch.float64),
           torch.full((D,), -1, **i32), torch.empty(cap, **i32), torch.empty(cap, dtype=torch.float32))
    idf_c = idf.to("cpu", torch.float64) if idf is not None else None
    _launch(native.lib(), sub, spec, sub_flags, idf_c, lr, trees, out, torch.device("cpu"))
    nnz, ntok, raw, status, idx, val = out
    if torch.any(status != STATUS_OK):
        raise RuntimeError("host featurizer failed on fallback documents")
    dev = res.nnz.device
    bad_t = torch.from_numpy(bad.astype(np.int64)).to(dev)
    res.nnz[bad_t] = nnz.to(dev)
    res.ntok[bad_t] = ntok.to(dev)
    res.raw[bad_t] = raw.to(dev)
    res.status[bad_t] = status.to(dev)
    if want_csr:
        sub_base = csr_slots(sub.offsets[:-1], torch.arange(D, dtype=torch.int64))
        n64 = nnz.to(torch.int64)
        total = int(n64.sum())
        if total:
            ptr = torch.zeros(D + 1, dtype=torch.int64)
            torch.cumsum(n64, 0, out=ptr[1:])
            row = torch.repeat_interleave(torch.arange(D), n64)
            within = torch.arange(total) - ptr[row]
            src = sub_base[row] + within
            dst = res.base[bad_t].cpu()[row] + within
            res.idx[dst.to(dev)] = idx[src].to(dev)
            res.val[dst.to(dev)] = val[src].to(dev)


# ------------------------------------------------------------------ CountVectorizer fit (K-05)
def _text_flags(spec: FeatureSpec) -> int:
    return (FLAG_CLEAN if spec.clean else 0) | (FLAG_STOPWORDS if spec.stopwords else 0)


def token_keys(text: PackedText, spec: FeatureSpec, device=None) -> tuple:
    """64-bit key of every token kept by clean -> tokenize -> stop-word removal, in document order:
    (keys int64 [T], ntok int64 [D]) on ``device``. Key = murmur3_x86_32(token, 42) << 32 |
    murmur3_x86_32(token, 0x9747b28c). Two passes of the fused text kernel (count, then write at
    the scanned offsets); documents the device path flags (too long / non-ASCII without cleaning)
    are redone on the host path."""
    C = native.lib()
    device = torch.device(device) if device is not None else text.device
    host_text = text
    text = text.to(device, non_blocking=True)
    D = len(text)
    st = spec.stop_table()
    stop = st.tensors(device) if st else None
    flags = _text_flags(spec)
    i32 = dict(dtype=torch.int32, device=device)
    ntok, status = torch.zeros(D, **i32), torch.full((D,), -1, **i32)
    C.token_keys(text.data, text.offsets, flags, stop, ntok, status, None, None, None, 0)
    bad = torch.nonzero(status != STATUS_OK).flatten().cpu().numpy() if D else np.zeros(0, np.int64)
    sub = sub_ntok = None
    if bad.size:
        strings = host_text.strings()
        sub = PackedText.from_strings([(strings[int(i)] or "") if spec.clean else (strings[int(i)] or "").lower()
                                       for i in bad])
        sub_flags = flags | (0 if spec.clean else FLAG_PRELOWERED)
        sub_ntok, sub_status = torch.zeros(len(bad), dtype=torch.int32), torch.full((len(bad),), -1, dtype=torch.int32)
        stop_c = st.tensors(torch.device("cpu")) if st else None
        C.token_keys(sub.data, sub.offsets, sub_flags, stop_c, sub_ntok, sub_status, None, None, None, 0)
        ntok[torch.from_numpy(bad).to(device)] = sub_ntok.to(device)
    n64 = ntok.to(torch.int64)
    key_off = torch.zeros(D + 1, dtype=torch.int64, device=device)
    torch.cumsum(n64, 0, out=key_off[1:])
    keys = torch.empty(int(key_off[-1]) if D else 0, dtype=torch.int64, device=device)
    status.fill_(-1)
    C.token_keys(text.data, text.offsets, flags, stop, ntok, status, key_off, keys, None, 0)
    if bad.size:
        sub_off = torch.zeros(len(bad) + 1, dtype=torch.int64)
        torch.cumsum(sub_ntok.to(torch.int64), 0, out=sub_off[1:])
        sub_keys = torch.empty(int(sub_off[-1]), dtype=torch.int64)
        C.token_keys(sub.data, sub.offsets, sub_flags, stop_c, sub_ntok, sub_status, sub_off, sub_keys, None, 0)
        ko = key_off.cpu()
        for j, i in enumerate(bad):
            a, b = int(sub_off[j]), int(sub_off[j + 1])
            keys[int(ko[i]): int(ko[i]) + (b - a)] = sub_keys[a:b].to(device)
    return keys, n64


def token_key(token: str) -> int:
    """Host value of the device token key (for mapping keys back to strings), as signed int64."""
    from . import oracle

    b = token.encode("utf-8")
    k = (oracle.murmur3_x86_32(b, 42) << 32) | oracle.murmur3_x86_32(b, 0x9747B28C)
    return k - (1 << 64) if k >= (1 << 63) else k


def term_doc_counts(keys: torch.Tensor, ntok: torch.Tensor) -> tuple:
    """Distinct keys with corpus term count and document frequency (sorted by key)."""
    dev = keys.device
    D = int(ntok.numel())
    if keys.numel() == 0:
        z = torch.zeros(0, dtype=torch.int64, device=dev)
        return z, z, z, z
    uk, inv, tf = torch.unique(keys, sorted=True, return_inverse=True, return_counts=True)
    doc = torch.repeat_interleave(torch.arange(D, device=dev, dtype=torch.int64), ntok, output_size=keys.numel())
    pairs = torch.unique(doc * uk.numel() + inv)          # distinct (doc, term)
    df = torch.bincount(pairs % uk.numel(), minlength=uk.numel())
    # first document of every term (to recover its string)
    first_doc = torch.full((uk.numel(),), D, dtype=torch.int64, device=dev)
    first_doc.scatter_reduce_(0, inv, doc, reduce="amin")
    return uk, tf, df, first_doc
