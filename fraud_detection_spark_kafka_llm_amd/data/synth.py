"""Synthetic scam / non-scam phone dialogues (stand-in for the missing BothBosu
``agent_conversation_all.csv``).

Schema matches the reference CSV (``dialogue, personality, type, labels``;
/root/reference/fraud_detection_spark.py:32-37). Dialogues alternate ``Innocent:`` / ``Suspect:``
turns like the real data (the df=numDocs buckets of ``innocent``/``suspect``/``hello`` in the
shipped IDF confirm the tags). Word choice mixes a shared conversational
vocabulary with class-specific lexicons seeded from the reference's reported top features
(PDF Tables VII-VIII: ``process, scheduled, insurance, social, prize, legitimate, security,
verify, identity, ...``); a small fraction of dialogues are deliberately low-signal so a depth-5
tree does not reach 100% — mirroring the reference's ~98% test accuracy.

Generation is fully vectorised in torch (byte-level gather), deterministic in ``seed``, and runs
on the GPU for the 10M-row benchmark configuration.
"""
from __future__ import annotations

import functools
from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

from ..ops.text import PAD, PackedText

COMMON = """hello hi yes no okay ok sure thanks thank you please well um uh so and the a to of in for on with
this that is it was be are have has i me my we our your can could would will just what when where how why
who call calling called phone today now time day week number name help sorry right good great fine really
know think need want like get got see let talk speak understand mean sir maam mr mrs moment minute
again sorry hear hold line back there here about from just also still very much more any some all""".split()

SCAM = """verify account security social urgent immediately suspended fraud fraudulent legal action arrest
warrant gift card wire transfer payment pay fee fine penalty irs tax refund prize won winner lottery claim
confirm identity information password pin code onetime otp detected suspicious activity compromised
legitimate assure officer agent department government administration bank credit card expire locked
remote access device computer virus install software download link click process processing scheduled
insurance premium policy benefits medicare consequences deactivated reference case badge transfer
bitcoin crypto investment guaranteed returns limited offer act fast secret confidential supervisor""".split()

BENIGN = """appointment reminder confirm delivery package order shipped tracking reservation table dinner
restaurant doctor dentist office clinic prescription pharmacy refill schedule reschedule tuesday
wednesday thursday friday monday weekend morning afternoon evening pm am meeting school teacher parent
conference survey feedback customer service satisfaction subscription renewal library book due return
plumber repair technician visit estimate quote neighbor party birthday invitation weather flight gate
checkin hotel booking balance statement question recipe catalog volunteer charity event tickets concert""".split()

TAGS = ["Innocent:", "Suspect:"]


@functools.lru_cache(maxsize=4)
def _tail_words(n: int = 30000, seed: int = 7) -> list:
    """Deterministic long-tail pseudo-words (names, places, rare terms) from syllables; the first
    30,000 are the same for every ``n`` (a wider vocabulary extends the default one)."""
    if n > 30000 and seed == 7:
        base = _tail_words(30000, 7)
        return base + _more_words(n - len(base), set(base))
    rng = np.random.default_rng(seed)
    syl = ["ka", "lo", "mi", "ren", "sta", "vi", "dor", "el", "an", "tor", "bri", "qu", "zen", "mar", "po",
           "li", "son", "ber", "ga", "ni", "ro", "che", "ty", "wen", "ha", "lu", "fe", "dra", "is", "om"]
    out, seen = [], set()
    while len(out) < n:
        w = "".join(syl[i] for i in rng.integers(0, len(syl), rng.integers(2, 5)))
        if w not in seen:
            seen.add(w)
            out.append(w)
    return out


def _more_words(n: int, seen: set) -> list:
    """``n`` further distinct pseudo-words (6-9 syllables from a wider syllable set)."""
    rng = np.random.default_rng(1234)
    syl = np.array(["ka", "lo", "mi", "ren", "sta", "vi", "dor", "el", "an", "tor", "bri", "qu", "zen", "mar",
                    "po", "li", "son", "ber", "ga", "ni", "ro", "che", "ty", "wen", "ha", "lu", "fe", "dra", "is",
                    "om", "xu", "jo", "pe", "sku", "ta", "vo", "gri", "ny", "bo", "ze"])
    out = []
    while len(out) < n:
        k = max(2 * (n - len(out)), 1024)
        lens = rng.integers(6, 10, k)
        picks = rng.integers(0, len(syl), (k, 9))
        for row, ln in zip(picks, lens):
            w = "".join(syl[row[:ln]])
            if w not in seen:
                seen.add(w)
                out.append(w)
                if len(out) == n:
                    break
    return out


TAIL = _tail_words()
SEPS = [" ", " ", " ", " ", ". ", ", ", "  ", "? ", "! ", ".  "]
PERSONALITIES = ["aggressive", "polite", "confused", "suspicious", "friendly", "neutral"]
TYPES = ["ssn", "bank", "prize", "tech support", "irs", "delivery", "appointment", "survey", "other"]


@dataclass
class SynthConfig:
    n: int = 1600
    seed: int = 42
    min_words: int = 150
    max_words: int = 450
    turn_len: int = 24          # words per speaker turn
    p_class_word: float = 0.10  # probability a word comes from the doc's class lexicon
    p_other_word: float = 0.012  # cross-class noise
    p_hard: float = 0.03        # fraction of low-signal dialogues
    hard_scale: float = 0.03
    p_tail: float = 0.12        # long-tail vocabulary share (sets the feature-space width)
    tail_words: int = 30000     # long-tail vocabulary size: 30K -> ~28K active of 2^18 buckets at
                                # 10M rows; 1M -> >200K active (a realistic wide vocabulary)


class _Vocab:
    def __init__(self, device, tail_words: int = 30000):
        tail = TAIL if tail_words == len(TAIL) else _tail_words(tail_words)
        words = TAGS + COMMON + SCAM + BENIGN + tail
        enc = [w.encode() for w in words]
        self.n_tags, self.n_common, self.n_scam, self.n_benign = len(TAGS), len(COMMON), len(SCAM), len(BENIGN)
        self.n_tail = len(tail)
        lens = torch.tensor([len(b) for b in enc], dtype=torch.int64)
        self.lens = lens.to(device)
        self.off = torch.cat([torch.zeros(1, dtype=torch.int64), torch.cumsum(lens, 0)[:-1]]).to(device)
        self.bytes = torch.from_numpy(np.frombuffer(b"".join(enc), dtype=np.uint8).copy()).to(device)
        senc = [s.encode() for s in SEPS]
        self.sep_lens = torch.tensor([len(b) for b in senc], dtype=torch.int64, device=device)
        self.sep_off = torch.cat([torch.zeros(1, dtype=torch.int64), torch.cumsum(self.sep_lens.cpu(), 0)[:-1]]).to(device)
        self.sep_bytes = torch.from_numpy(np.frombuffer(b"".join(senc), dtype=np.uint8).copy()).to(device)


_VOCABS: dict = {}


def _vocab(device: torch.device, tail_words: int) -> _Vocab:
    key = (str(device), tail_words)
    if key not in _VOCABS:
        _VOCABS[key] = _Vocab(device, tail_words)
    return _VOCABS[key]


def generate(cfg: SynthConfig = SynthConfig(), device="cpu", start: int = 0) -> tuple[PackedText, torch.Tensor]:
    """Generate dialogues ``start .. start+n`` of the stream seeded by ``cfg.seed``.

    Returns (PackedText on ``device``, labels float64 [n]). ``(seed, start)`` identifies a chunk:
    large corpora are generated as chunks with distinct ``start`` values (independent streams),
    and the same (seed, start, n) always yields identical bytes on any device.
    """
    device = torch.device(device)
    V = _vocab(device, cfg.tail_words)
    n = cfg.n
    g = torch.Generator(device="cpu").manual_seed(int(cfg.seed) * 1_000_003 + int(start))
    # per-doc draws (host RNG for determinism across devices; tiny)
    labels = (torch.rand(n, generator=g) < 0.5).to(torch.int64)
    nwords = torch.randint(cfg.min_words, cfg.max_words + 1, (n,), generator=g)
    hard = torch.rand(n, generator=g) < cfg.p_hard
    tag0 = torch.randint(0, 2, (n,), generator=g)
    seed_dev = int(torch.randint(0, 2**62, (1,), generator=g))
    labels, nwords, hard, tag0 = labels.to(device), nwords.to(device), hard.to(device), tag0.to(device)

    W = int(nwords.sum())
    doc = torch.repeat_interleave(torch.arange(n, device=device), nwords, output_size=W)
    starts = torch.cumsum(nwords, 0) - nwords
    pos = torch.arange(W, device=device) - starts[doc]
    gd = torch.Generator(device=device).manual_seed(seed_dev)
    u = torch.rand(W, generator=gd, device=device)
    pick = torch.rand(W, generator=gd, device=device)
    sep = torch.randint(0, len(SEPS), (W,), generator=gd, device=device)

    doc_scale = torch.where(hard, torch.full((n,), cfg.hard_scale, device=device), torch.ones(n, device=device))
    scale = doc_scale[doc]
    p_cls = cfg.p_class_word * scale
    p_oth = cfg.p_other_word * torch.ones_like(u)
    is_scam = labels[doc] == 1
    base_c = V.n_tags
    base_s = base_c + V.n_common
    base_b = base_s + V.n_scam
    # Zipf-ish choice inside each lexicon: floor(len * pick^2)
    zc = (pick * pick * V.n_common).to(torch.int64).clamp_max(V.n_common - 1)
    # own-class cue words are Zipfian (a few dominant cues, like the reference's top features);
    # cross-class noise is uniform so the dominant cues stay discriminative
    p3 = pick.pow(3)
    zs = (p3 * V.n_scam).to(torch.int64).clamp_max(V.n_scam - 1)
    zb = (p3 * V.n_benign).to(torch.int64).clamp_max(V.n_benign - 1)
    us = (pick * V.n_scam).to(torch.int64).clamp_max(V.n_scam - 1)
    ub = (pick * V.n_benign).to(torch.int64).clamp_max(V.n_benign - 1)
    base_t = base_b + V.n_benign
    zt = (p3 * V.n_tail).to(torch.int64).clamp_max(V.n_tail - 1)
    own = torch.where(is_scam, base_s + zs, base_b + zb)
    other = torch.where(is_scam, base_b + ub, base_s + us)
    word = torch.where(u < p_cls, own, torch.where(u < p_cls + p_oth, other,
                       torch.where(u > 1.0 - cfg.p_tail, base_t + zt, base_c + zc)))
    tag_here = (pos % cfg.turn_len) == 0
    word = torch.where(tag_here, ((pos // cfg.turn_len + tag0[doc]) % 2), word)
    sep = torch.where(tag_here, torch.zeros_like(sep), sep)
    last = pos == (nwords[doc] - 1)
    sep = torch.where(last, torch.full_like(sep, 4), sep)    # end with ". "

    tok_len = V.lens[word] + V.sep_lens[sep]
    doc_bytes = torch.zeros(n, dtype=torch.int64, device=device).index_add_(0, doc, tok_len)
    offsets = torch.zeros(n + 1, dtype=torch.int64, device=device)
    torch.cumsum(doc_bytes, 0, out=offsets[1:])
    total = int(offsets[-1])
    data = torch.zeros(total + PAD, dtype=torch.uint8, device=device)
    tok_start = torch.cumsum(tok_len, 0) - tok_len
    # bytes of the word part
    wl = V.lens[word]
    Bw = int(wl.sum())
    t_of = torch.repeat_interleave(torch.arange(W, device=device), wl, output_size=Bw)
    within = torch.arange(Bw, device=device) - (torch.cumsum(wl, 0) - wl)[t_of]
    data[tok_start[t_of] + within] = V.bytes[V.off[word][t_of] + within]
    # bytes of the separator part
    sl = V.sep_lens[sep]
    Bs = int(sl.sum())
    t_of = torch.repeat_interleave(torch.arange(W, device=device), sl, output_size=Bs)
    within = torch.arange(Bs, device=device) - (torch.cumsum(sl, 0) - sl)[t_of]
    data[tok_start[t_of] + wl[t_of] + within] = V.sep_bytes[V.sep_off[sep][t_of] + within]
    return PackedText(data, offsets), labels.to(torch.float64)


def generate_frame(cfg: SynthConfig = SynthConfig()):
    """A ``Frame`` with the reference CSV schema (labels as strings like the raw CSV)."""
    from ..ml.frame import Frame, TextColumn

    text, labels = generate(cfg, "cpu")
    rng = np.random.default_rng(cfg.seed)
    strings = text.strings()
    lab = labels.numpy().astype(int)
    types = [TYPES[rng.integers(0, 6)] if y else TYPES[rng.integers(6, len(TYPES))] for y in lab]
    pers = [PERSONALITIES[i] for i in rng.integers(0, len(PERSONALITIES), len(lab))]
    return Frame({"dialogue": TextColumn(strings), "personality": pers, "type": types,
                  "labels": [str(y) for y in lab]}, ["dialogue", "personality", "type", "labels"])


def to_csv(path: str, cfg: SynthConfig = SynthConfig()) -> None:
    generate_frame(cfg).toPandas().to_csv(path, index=False)
