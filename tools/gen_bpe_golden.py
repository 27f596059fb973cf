"""Golden vectors for clipmi.tokenizer (dataset.py:152-159).

The reference tokenises captions with CLIPProcessor(text=..., padding="max_length", max_length=77,
truncation=True); its vocab.json / merges.txt are hub downloads, absent offline.  This script
trains a small CLIP-style byte-level BPE (vocabulary layout as openai/clip-vit-*: the 256 byte
symbols, the same with "</w>", the merged tokens in merge order, then <|startoftext|> and
<|endoftext|>) on a synthetic caption corpus, writes it to tests/golden/bpe/, and records the ids
and attention masks that transformers.CLIPTokenizer (the reference's tokenizer class) produces on
the same files for a set of captions chosen to hit the pipeline's edge cases.

  python tools/gen_bpe_golden.py   (CPU; needs transformers + tokenizers, both in this image)
"""
import json
import os
import random
from collections import Counter

import numpy as np

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "bpe")

WORDS = ("a person who looks happy smiling joyful face with bright eyes the man woman child is feeling sad "
         "angry surprised fearful disgusted neutral calm excited nervous anxious peaceful content tired "
         "bored confused proud ashamed lonely hopeful photo of an expression showing emotion emotional "
         "their body language suggests that they are in a state of deep sorrow or intense happiness and "
         "relaxed posture tense shoulders furrowed brows wide open mouth tears laughing crying yelling "
         "quietly sitting standing walking outdoors indoors scene people group together alone").split()


def corpus(rng, n=3000):
    out = []
    for _ in range(n):
        k = rng.randint(3, 14)
        s = " ".join(rng.choice(WORDS) for _ in range(k))
        if rng.random() < 0.3:
            s = s.capitalize() + rng.choice([".", "!", "?", ",", "..."])
        if rng.random() < 0.1:
            s += f" {rng.randint(0, 99)}"
        out.append(s)
    return out


def train(lines, n_merges=600):
    from clipmi.tokenizer import CLIPTokenizer, bytes_to_unicode
    be = bytes_to_unicode()
    base = list(be.values())
    vocab_list = base + [c + "</w>" for c in base]
    # word frequencies after the CLIP normalizer / pre-tokenizer (pre_tokenize needs an instance)
    stub = CLIPTokenizer({**{t: i for i, t in enumerate(vocab_list)}, "<|startoftext|>": len(vocab_list),
                          "<|endoftext|>": len(vocab_list) + 1}, [])
    freq = Counter()
    for ln in lines:
        freq.update(stub.pre_tokenize(stub.normalize(ln)))
    words = {w: (list(w[:-1]) + [w[-1] + "</w>"]) for w in freq}
    merges = []
    for _ in range(n_merges):
        pairs = Counter()
        for w, f in freq.items():
            s = words[w]
            for i in range(len(s) - 1):
                pairs[(s[i], s[i + 1])] += f
        if not pairs:
            break
        (a, b), c = max(pairs.items(), key=lambda kv: (kv[1], kv[0]))
        if c < 2:
            break
        merges.append((a, b))
        for w in freq:
            s = words[w]
            i, t = 0, []
            while i < len(s):
                if i + 1 < len(s) and s[i] == a and s[i + 1] == b:
                    t.append(a + b)
                    i += 2
                else:
                    t.append(s[i])
                    i += 1
            words[w] = t
    for a, b in merges:
        if a + b not in vocab_list:
            vocab_list.append(a + b)
    vocab_list += ["<|startoftext|>", "<|endoftext|>"]
    return {t: i for i, t in enumerate(vocab_list)}, merges


CASES = [
    "a photo of a happy person",
    "",
    "   ",
    "The Man is SMILING!!!",
    "She's feeling sad, isn't she? They'll be fine; we'd go. I'm here, you've won.",
    "emotion   with\tmultiple\n\nspaces and\r\nnewlines",
    "numbers 12345 and 3.14 and 1,000,000",
    "Café naïve résumé — “quoted” ‘text’ …",
    "unicode: 日本語のテキスト 😀 🎉 ñ ß Ω",
    "Straße İstanbul ǅemal",  # case mapping edge cases
    "<|startoftext|>literal special tokens<|endoftext|> inside",
    "punctuation runs ?!?! ... --- ### @@@ (parens) [brackets] {braces}",
    "a" * 200,
    " ".join(["happiness"] * 120),  # truncation: far more than 75 tokens
    "word " * 74 + "end",  # exactly around the 75-token boundary
    "Mixed-CASE hyphenated-words and under_scores and e-mail@example.com",
    "xyzzy qwerty zzz unknownwords",  # mostly unmerged symbols
    " non-breaking em-space　ideographic",
]


def main():
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "vlm-clip_amd"))
    from transformers import CLIPTokenizer as HFCLIPTokenizer
    rng = random.Random(1234)
    vocab, merges = train(corpus(rng))
    os.makedirs(OUT, exist_ok=True)
    with open(os.path.join(OUT, "vocab.json"), "w", encoding="utf-8") as f:
        json.dump(vocab, f, ensure_ascii=False)
    with open(os.path.join(OUT, "merges.txt"), "w", encoding="utf-8") as f:
        f.write("#version: 0.2\n")
        for a, b in merges:
            f.write(f"{a} {b}\n")
    hf = HFCLIPTokenizer(vocab=vocab, merges=[(a, b) for a, b in merges])
    cases = CASES + corpus(random.Random(99), 40)
    enc = hf(cases, padding="max_length", max_length=77, truncation=True, return_tensors="np")
    # batch-1 form too (the dataset calls the processor per caption)
    one = hf(cases[0], padding="max_length", max_length=77, truncation=True, return_tensors="np")
    assert np.array_equal(one["input_ids"][0], enc["input_ids"][0])
    with open(os.path.join(OUT, "captions.json"), "w", encoding="utf-8") as f:
        json.dump(cases, f, ensure_ascii=False, indent=0)
    np.savez_compressed(os.path.join(OUT, "ids.npz"), input_ids=enc["input_ids"].astype(np.int32),
                        attention_mask=enc["attention_mask"].astype(np.int8))
    print(f"vocab {len(vocab)}, merges {len(merges)}, cases {len(cases)} -> {OUT}")


if __name__ == "__main__":
    main()
