"""Undo PTB / WikiText tokenisation artefacts before re-tokenising
(reference tasks/zeroshot_gpt/detokenizer.py; same rules)."""
import re

_WIKI_SUBS = [("s '", "s'"), (" @-@ ", "-"), (" @,@ ", ","), (" @.@ ", "."), (" : ", ": "),
              (" ; ", "; "), (" . ", ". "), (" ! ", "! "), (" ? ", "? "), (" , ", ", ")]
_WIKI_RE = [(r"/' [0-9]/", r"/'[0-9]/"), (r"\(\s*([^\)]*?)\s*\)", r"(\1)"),
            (r"\[\s*([^\]]*?)\s*\]", r"[\1]"), (r"{\s*([^}]*?)\s*}", r"{\1}"),
            (r"\"\s*([^\"]*?)\s*\"", r'"\1"'), (r"'\s*([^']*?)\s*'", r"'\1'")]
_WIKI_TAIL = [("= = = =", "===="), ("= = =", "==="), ("= =", "=="),
              (" " + chr(176) + " ", chr(176)), (" \n", "\n"), ("\n ", "\n"), (" N ", " 1 "),
              (" 's", "'s")]


def ptb_detokenizer(s):
    for a, b in ((" '", "'"), (" \n", "\n"), ("\n ", "\n"), (" n't", "n't"), (" N ", "1 "),
                 ("$ 1", "$1"), ("# 1", "#1")):
        s = s.replace(a, b)
    return s


def wikitext_detokenizer(s):
    s = s.replace(*_WIKI_SUBS[0])
    s = re.sub(*_WIKI_RE[0], s)
    for a, b in _WIKI_SUBS[1:]:
        s = s.replace(a, b)
    for pat, rep in _WIKI_RE[1:]:
        s = re.sub(pat, rep, s)
    for a, b in _WIKI_TAIL:
        s = s.replace(a, b)
    return s


def lambada_detokenizer(s):
    return s


_DETOKENIZERS = {"ptb": ptb_detokenizer, "wiki": wikitext_detokenizer,
                 "lambada": lambada_detokenizer}


def get_detokenizer(path):
    for key, fn in _DETOKENIZERS.items():
        if key in path:
            return fn
    return lambda s: s
