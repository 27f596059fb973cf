"""CLIP byte-level BPE tokenizer: the caption half of the reference's input step.

dataset.py:152-159 (/root/reference/dataset.py) tokenises every caption through
``CLIPProcessor(text=caption, padding="max_length", max_length=77, truncation=True)``, i.e. the
``tokenizers``-backed ``transformers.CLIPTokenizer`` (transformers 5.x,
models/clip/tokenization_clip.py).  This module restates that pipeline over caller-supplied
``vocab.json`` / ``merges.txt`` (the hub files are downloads; none ship offline):

  1. special tokens (``<|startoftext|>``, ``<|endoftext|>``) are split out of the raw text first;
  2. normalizer: NFC, every whitespace run -> one space, lowercase;
  3. pre-tokenizer: the CLIP split regex (matches kept, the rest dropped), then the GPT-2
     byte-level regex and byte -> unicode mapping (``add_prefix_space=False``);
  4. BPE with ``end_of_word_suffix="</w>"``: the word's last symbol carries the suffix, symbols not
     in the vocabulary become the unknown token (not fused), merges applied lowest rank first,
     leftmost first among equal ranks (the ``tokenizers`` heap order);
  5. post-processor: ``<|startoftext|> ids <|endoftext|>``; truncation keeps the first
     ``max_length - 2`` ids; padding to ``max_length`` with ``<|endoftext|>`` and mask 0.

Pinned by tests/golden/bpe/ (ids produced by transformers.CLIPTokenizer on the same files).
This is host-side input preparation, as in the reference (its data loader runs on the CPU); the
ids then go to the device like the reference's ``input_ids``.
"""
from __future__ import annotations

import heapq
import json
import unicodedata

import numpy as np
import regex

_CLIP_SPLIT = regex.compile(
    r"""<\|startoftext\|>|<\|endoftext\|>|'s|'t|'re|'ve|'m|'ll|'d|[\p{L}]+|[\p{N}]|[^\s\p{L}\p{N}]+""")
_GPT2_SPLIT = regex.compile(r"""'s|'t|'re|'ve|'m|'ll|'d| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|\s+(?!\S)|\s+""")
_WS = regex.compile(r"\s+")


def bytes_to_unicode():
    """The byte-level alphabet: printable latin-1 bytes map to themselves, the rest to 256+."""
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + \
        list(range(ord("®"), ord("ÿ") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return dict(zip(bs, (chr(c) for c in cs)))


class CLIPTokenizer:
    """Mirror of ``transformers.CLIPTokenizer``'s call interface for the reference's use."""

    model_input_names = ["input_ids", "attention_mask"]

    def __init__(self, vocab, merges, unk_token="<|endoftext|>", bos_token="<|startoftext|>",
                 eos_token="<|endoftext|>", pad_token="<|endoftext|>"):
        if isinstance(vocab, str):
            with open(vocab, encoding="utf-8") as f:
                vocab = json.load(f)
        if isinstance(merges, str):
            with open(merges, encoding="utf-8") as f:
                merges = [ln.rstrip("\n") for ln in f]
            merges = [m for m in merges if m and not m.startswith("#version")]
        self.vocab = dict(vocab)
        self.unk_token, self.bos_token, self.eos_token, self.pad_token = unk_token, bos_token, eos_token, pad_token
        for t in (unk_token, bos_token, eos_token, pad_token):
            if t not in self.vocab:
                raise ValueError(f"special token {t!r} missing from the vocabulary")
        self.unk_token_id = self.vocab[unk_token]
        self.bos_token_id = self.vocab[bos_token]
        self.eos_token_id = self.vocab[eos_token]
        self.pad_token_id = self.vocab[pad_token]
        self.specials = {t: self.vocab[t] for t in (bos_token, eos_token, unk_token, pad_token)}
        self._special_re = regex.compile("|".join(regex.escape(t) for t in sorted(self.specials, key=len, reverse=True)))
        # merges: (left id, right id) -> (rank, merged id)
        self.merges = {}
        for rank, m in enumerate(merges):
            parts = m.split(" ") if isinstance(m, str) else list(m)
            if len(parts) != 2:
                raise ValueError(f"bad merge line {m!r}")
            a, b = parts
            if a not in self.vocab or b not in self.vocab or a + b not in self.vocab:
                raise ValueError(f"merge {m!r} refers to a token missing from the vocabulary")
            self.merges.setdefault((self.vocab[a], self.vocab[b]), (rank, self.vocab[a + b]))
        self.byte_encoder = bytes_to_unicode()
        self._cache = {}

    @classmethod
    def from_files(cls, vocab_file, merges_file, **kw):
        return cls(vocab_file, merges_file, **kw)

    # ------------------------------------------------------------------ pipeline pieces
    @staticmethod
    def normalize(text):
        return _WS.sub(" ", unicodedata.normalize("NFC", text)).lower()

    def pre_tokenize(self, text):
        words = []
        for piece in _CLIP_SPLIT.findall(text):
            for w in _GPT2_SPLIT.findall(piece):
                words.append("".join(self.byte_encoder[b] for b in w.encode("utf-8")))
        return words

    def bpe(self, word):
        """ids of one pre-tokenized word (byte-level unicode string)."""
        hit = self._cache.get(word)
        if hit is not None:
            return hit
        chars = list(word)
        chars[-1] = chars[-1] + "</w>"
        sym = [self.vocab.get(c, self.unk_token_id) for c in chars]
        n = len(sym)
        nxt = list(range(1, n + 1))
        prv = list(range(-1, n - 1))
        alive = [True] * n
        heap = []
        for i in range(n - 1):
            m = self.merges.get((sym[i], sym[i + 1]))
            if m is not None:
                heapq.heappush(heap, (m[0], i, sym[i], sym[i + 1]))
        while heap:
            rank, i, a, b = heapq.heappop(heap)
            j = nxt[i] if i < n else n
            if not alive[i] or j >= n or sym[i] != a or sym[j] != b:
                continue  # stale: a neighbour was merged since this pair was queued
            sym[i] = self.merges[(a, b)][1]
            alive[j] = False
            nxt[i] = nxt[j]
            if nxt[j] < n:
                prv[nxt[j]] = i
            p = prv[i]
            if p >= 0:
                m = self.merges.get((sym[p], sym[i]))
                if m is not None:
                    heapq.heappush(heap, (m[0], p, sym[p], sym[i]))
            q = nxt[i]
            if q < n:
                m = self.merges.get((sym[i], sym[q]))
                if m is not None:
                    heapq.heappush(heap, (m[0], i, sym[i], sym[q]))
        out = [sym[i] for i in range(n) if alive[i]]
        if len(self._cache) < 100000:
            self._cache[word] = out
        return out

    def encode(self, text, add_special_tokens=True):
        ids = []
        pos = 0
        for m in self._special_re.finditer(text):
            ids.extend(self._encode_plain(text[pos:m.start()]))
            ids.append(self.specials[m.group(0)])
            pos = m.end()
        ids.extend(self._encode_plain(text[pos:]))
        if add_special_tokens:
            ids = [self.bos_token_id] + ids + [self.eos_token_id]
        return ids

    def _encode_plain(self, text):
        out = []
        if text:
            for w in self.pre_tokenize(self.normalize(text)):
                out.extend(self.bpe(w))
        return out

    # ------------------------------------------------------------------ __call__
    def __call__(self, text, padding="max_length", max_length=77, truncation=True, return_tensors=None,
                 add_special_tokens=True):
        """dataset.py:152-159's call: returns {"input_ids", "attention_mask"} of shape [B, max_length]
        (B = 1 for a single string, as CLIPProcessor returns before the dataset's squeeze(0))."""
        texts = [text] if isinstance(text, str) else list(text)
        if padding not in ("max_length", True, "longest", False, "do_not_pad"):
            raise ValueError(f"unsupported padding {padding!r}")
        rows = []
        for t in texts:
            ids = self.encode(t, add_special_tokens=False)
            if truncation and max_length is not None:
                keep = max_length - (2 if add_special_tokens else 0)
                ids = ids[:max(0, keep)]
            if add_special_tokens:
                ids = [self.bos_token_id] + ids + [self.eos_token_id]
            rows.append(ids)
        if padding == "max_length":
            width = max_length
        elif padding in (True, "longest"):
            width = max(len(r) for r in rows) if rows else 0
        else:
            width = None
        if width is None:
            if return_tensors is not None and len({len(r) for r in rows}) > 1:
                raise ValueError("unpadded rows of different lengths cannot form a tensor")
            width = max(len(r) for r in rows) if rows else 0
        ids = np.full((len(rows), width), self.pad_token_id, dtype=np.int64)
        mask = np.zeros((len(rows), width), dtype=np.int64)
        for i, r in enumerate(rows):
            ids[i, :len(r)] = r
            mask[i, :len(r)] = 1
        if return_tensors == "pt":
            import torch
            return {"input_ids": torch.from_numpy(ids), "attention_mask": torch.from_numpy(mask)}
        if return_tensors == "np":
            return {"input_ids": ids, "attention_mask": mask}
        return {"input_ids": [r.tolist()[:len(rows[i])] if padding in (False, "do_not_pad") else r.tolist()
                              for i, r in enumerate(ids)],
                "attention_mask": [m.tolist()[:len(rows[i])] if padding in (False, "do_not_pad") else m.tolist()
                                   for i, m in enumerate(mask)]}
