"""Regex word tokenizer used for answer matching (the DPR ``SimpleTokenizer``
that reference ``tasks/orqa/unsupervised/tokenizers.py`` vendors): runs of
letters/digits/marks, or any single non-space non-control character."""
import regex


class Tokens:
    def __init__(self, words):
        self._words = words

    def __len__(self):
        return len(self._words)

    def words(self, uncased=False):
        return [w.lower() for w in self._words] if uncased else list(self._words)


class SimpleTokenizer:
    ALPHA_NUM = r"[\p{L}\p{N}\p{M}]+"
    NON_WS = r"[^\p{Z}\p{C}]"

    def __init__(self, **kwargs):
        self._regexp = regex.compile(f"({self.ALPHA_NUM})|({self.NON_WS})",
                                     flags=regex.IGNORECASE + regex.UNICODE + regex.MULTILINE)

    def tokenize(self, text):
        return Tokens([m.group() for m in self._regexp.finditer(text)])
