"""Dialogues over 64 KB on the device: segment, featurize per segment, merge, score (K-01..K-07).

The fused featurize+score kernel keeps one dialogue's cleaned bytes and tokens in LDS (64 KB /
16384 tokens on the long-dialogue variant). Longer transcripts are cut at raw positions ``p`` with
``raw[p] == ' '`` and ``raw[p-1]`` an ASCII letter, into segments of at most ``SEG_BYTES`` bytes
that keep the separator as their last byte. Cleaning is per byte (a multi-byte UTF-8 sequence
never spans such a cut), and a segment ending in "<letter><space>" tokenizes exactly like that
stretch of the whole dialogue (Spark's ``split("\\\\s")`` drops only the trailing empty piece
that the separator creates), so the dialogue's term counts are the sums of its segments' counts.

Segments are contiguous in the dialogue's buffer, so they run as a ``doc_list`` launch of the
long-dialogue kernel straight from the device copy of the text (no host re-pack). Per-segment
(bucket, count) CSR rows are merged per dialogue (sort + segment sum), multiplied by the IDF and
scored by the same native CSR scorer whose lane-strided order equals the fused kernel's, so the
result is bitwise equal to the host featurizer's whole-dialogue result. Dialogues without a
valid cut inside a window (one "word" longer than a segment) are left to the host path.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch

SEG_BYTES = 16000      # <= 16001 tokens per segment: fits the long kernel's 16384-token LDS table


def split_points(buf: np.ndarray, s: int, e: int, seg: int = SEG_BYTES) -> Optional[np.ndarray]:
    """Boundaries ``[s, c1, ..., e]`` of the segments of ``buf[s:e]`` (each ``<= seg`` bytes; every
    inner boundary follows a space preceded by an ASCII letter), or None if there is no such cut."""
    if e - s <= seg:
        return np.array([s, e], dtype=np.int64)
    a = buf[s:e]
    letter = ((a[:-1] | 0x20) >= ord("a")) & ((a[:-1] | 0x20) <= ord("z"))
    cuts = np.flatnonzero((a[1:] == 0x20) & letter) + 2          # relative end (exclusive) after the space
    out = [s]
    pos = 0
    n = e - s
    while n - pos > seg:
        k = int(np.searchsorted(cuts, pos + seg, side="right")) - 1
        if k < 0 or cuts[k] <= pos:
            return None
        pos = int(cuts[k])
        out.append(s + pos)
    out.append(e)
    return np.asarray(out, dtype=np.int64)


def featurize_long(data_dev: torch.Tensor, host_buf: np.ndarray, doc_off: np.ndarray, docs: np.ndarray, spec,
                   idf_t: Optional[torch.Tensor], lr, trees, device):
    """Score dialogues ``docs`` (indices into ``doc_off``) whose bytes are ``data_dev`` (device)
    and ``host_buf`` (the same bytes on the host, for the cut search).

    Returns ``(done, raw, nnz, ntok, csr)``: ``done`` bool [len(docs)] (False: left to the host),
    ``raw`` [n_done, K] fp64 on ``device``, ``nnz``/``ntok`` int32 [n_done], and ``csr`` =
    (indptr int64 [n_done+1], idx int32, val fp64) of the merged rows."""
    from . import native
    from .sparse import score_csr
    from ..ml.linalg import VectorColumn
    from .text import FLAG_BINARY, FLAG_WRITE_CSR, STATUS_OK, _flags, csr_capacity, csr_slots

    C = native.lib()
    bounds, seg_doc, done = [], [], np.zeros(len(docs), dtype=bool)
    for j, d in enumerate(docs):
        b = split_points(host_buf, int(doc_off[d]), int(doc_off[d + 1]))
        if b is None:
            continue
        done[j] = True
        bounds.append(b)
        seg_doc.append(np.full(b.size - 1, j, dtype=np.int64))
    K = trees.K if trees is not None else 1
    empty = (done, torch.zeros((0, K), dtype=torch.float64, device=device), torch.zeros(0, dtype=torch.int32),
             torch.zeros(0, dtype=torch.int32), None)
    if not bounds:
        return empty
    # boundaries of all dialogues back to back; pseudo-documents between dialogues are skipped
    offs = np.concatenate(bounds)
    first = np.cumsum([0] + [b.size for b in bounds[:-1]])
    seg_idx = np.concatenate([f + np.arange(b.size - 1) for f, b in zip(first, bounds)]).astype(np.int32)
    seg_doc = np.concatenate(seg_doc)
    S = int(offs.size - 1)
    offs_t = torch.from_numpy(offs).to(device)
    list_t = torch.from_numpy(seg_idx).to(device)
    i32 = dict(dtype=torch.int32, device=device)
    nnz, ntok = torch.zeros(S, **i32), torch.zeros(S, **i32)
    status = torch.full((S,), -1, **i32)
    raw_dummy = torch.zeros((S, 1), dtype=torch.float64, device=device)
    cap = csr_capacity(int(data_dev.numel()), S)
    idx, val = torch.empty(cap, **i32), torch.empty(cap, dtype=torch.float32, device=device)
    flags = (_flags(spec, None, None, None, True) | FLAG_WRITE_CSR) & ~FLAG_BINARY   # raw term counts
    st, vt = spec.stop_table(), spec.vocab_table()
    C.featurize_score(data_dev, offs_t, flags, spec.dim, st.tensors(device) if st else None,
                      vt.tensors(device) if vt else None, 0.0, None, None, 0.0, None, 1,
                      idx, val, nnz, ntok, raw_dummy, status, None, 0, list_t)
    seg_status = status[list_t.long()].cpu().numpy()
    ok_doc = np.ones(len(docs), dtype=bool)
    ok_doc[seg_doc[seg_status != STATUS_OK]] = False
    done &= ok_doc
    keep_seg = done[seg_doc]
    if not keep_seg.any():
        return empty
    sel = torch.from_numpy(seg_idx[keep_seg].astype(np.int64)).to(device)
    sdoc_old = seg_doc[keep_seg]
    remap = np.cumsum(done) - 1                                  # dialogue j -> row of the done dialogues
    sdoc = torch.from_numpy(remap[sdoc_old]).to(device)
    n_done = int(done.sum())
    # gather every kept segment's CSR entries (written at csr_slots(segment start, segment index))
    cnt = nnz[sel].long()
    base = csr_slots(offs_t[sel], sel)
    total = int(cnt.sum())
    starts = torch.zeros(cnt.numel() + 1, dtype=torch.int64, device=device)
    torch.cumsum(cnt, 0, out=starts[1:])
    owner = torch.repeat_interleave(torch.arange(cnt.numel(), device=device), cnt, output_size=total)
    pos = base[owner] + (torch.arange(total, device=device) - starts[owner])
    feat = idx[pos].long()
    counts = val[pos].to(torch.float64)                          # exact integers (< 2^24)
    key = sdoc[owner] * int(spec.dim) + feat
    ukey, inv = torch.unique(key, sorted=True, return_inverse=True)
    summed = torch.zeros(ukey.numel(), dtype=torch.float64, device=device).index_add_(0, inv, counts)
    row = ukey // int(spec.dim)
    col = (ukey % int(spec.dim)).to(torch.int32)
    tok = torch.zeros(n_done, dtype=torch.int64, device=device).index_add_(0, sdoc, ntok[sel].long())
    if spec.vocab is not None and (spec.min_tf > 1.0 or 0.0 < spec.min_tf < 1.0):
        thr = torch.full_like(summed, float(spec.min_tf)) if spec.min_tf >= 1.0 else spec.min_tf * tok[row].double()
        k = summed >= thr
        row, col, summed = row[k], col[k], summed[k]
    if spec.binary:
        v = torch.ones_like(summed)
    else:
        v = summed
    if idf_t is not None:
        v = v * idf_t[col.long()]
    per = torch.bincount(row, minlength=n_done)
    indptr = torch.zeros(n_done + 1, dtype=torch.int64, device=device)
    torch.cumsum(per, 0, out=indptr[1:])
    vc = VectorColumn(int(spec.dim), indptr, col, v)
    scorer = lr if lr is not None else trees
    raw = score_csr(vc, scorer) if scorer is not None else torch.zeros((n_done, 1), dtype=torch.float64, device=device)
    return done, raw, per.to(torch.int32), tok.to(torch.int32), (indptr, col, v)
