"""CLIP BPE tokenizer (clipmi.tokenizer) vs the reference's tokenizer class.

dataset.py:152-159 tokenises captions through CLIPProcessor(..., padding="max_length",
max_length=77, truncation=True) = transformers.CLIPTokenizer.  tests/golden/bpe/ holds a CLIP-style
vocabulary trained offline and the ids/masks transformers.CLIPTokenizer produced from it
(tools/gen_bpe_golden.py); the live comparison runs when transformers is importable."""
import json
import os
import random

import numpy as np
import pytest

from clipmi.tokenizer import CLIPTokenizer

D = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "bpe")


@pytest.fixture(scope="module")
def tok():
    return CLIPTokenizer(os.path.join(D, "vocab.json"), os.path.join(D, "merges.txt"))


def test_matches_golden_ids(tok):
    caps = json.load(open(os.path.join(D, "captions.json"), encoding="utf-8"))
    g = np.load(os.path.join(D, "ids.npz"))
    out = tok(caps, padding="max_length", max_length=77, truncation=True, return_tensors="np")
    assert out["input_ids"].shape == (len(caps), 77)
    np.testing.assert_array_equal(out["input_ids"], g["input_ids"])
    np.testing.assert_array_equal(out["attention_mask"], g["attention_mask"])


def test_single_caption_and_torch_tensors(tok):
    torch = pytest.importorskip("torch")
    enc = tok("a photo of a happy person", padding="max_length", max_length=77, truncation=True,
              return_tensors="pt")
    assert enc["input_ids"].shape == (1, 77) and enc["input_ids"].dtype == torch.int64
    ids = enc["input_ids"][0]
    n = int(enc["attention_mask"][0].sum())
    assert ids[0] == tok.bos_token_id and ids[n - 1] == tok.eos_token_id
    assert (ids[n:] == tok.pad_token_id).all()


def test_truncation_keeps_bos_and_eos(tok):
    enc = tok(" ".join(["happiness"] * 200), padding="max_length", max_length=77, truncation=True,
              return_tensors="np")
    ids, m = enc["input_ids"][0], enc["attention_mask"][0]
    assert m.sum() == 77 and ids[0] == tok.bos_token_id and ids[-1] == tok.eos_token_id


def test_live_against_transformers(tok):
    tr = pytest.importorskip("transformers")
    vocab = json.load(open(os.path.join(D, "vocab.json"), encoding="utf-8"))
    merges = [tuple(ln.rstrip("\n").split(" ")) for ln in open(os.path.join(D, "merges.txt"), encoding="utf-8")
              if ln.strip() and not ln.startswith("#version")]
    hf = tr.CLIPTokenizer(vocab=vocab, merges=merges)
    rng = random.Random(7)
    alphabet = list("abcdefghijklmnopqrstuvwxyz ABCDEFGHIJ  0123456789.,!?'-’éüñß日本😀\t\n") + \
        ["happy ", "sad ", "'s ", "'ll ", "person ", "emotion ", "<|endoftext|>"]
    texts = ["".join(rng.choice(alphabet) for _ in range(rng.randint(0, 120))) for _ in range(300)]
    a = tok(texts, padding="max_length", max_length=77, truncation=True, return_tensors="np")
    b = hf(texts, padding="max_length", max_length=77, truncation=True, return_tensors="np")
    np.testing.assert_array_equal(a["input_ids"], b["input_ids"])
    np.testing.assert_array_equal(a["attention_mask"], b["attention_mask"])


def test_rejects_inconsistent_files():
    with pytest.raises(ValueError):
        CLIPTokenizer({"a": 0, "<|startoftext|>": 1, "<|endoftext|>": 2}, ["a b"])
    with pytest.raises(ValueError):
        CLIPTokenizer({"a": 0}, [])
