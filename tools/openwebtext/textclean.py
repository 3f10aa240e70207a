"""Shared helpers for the corpus-cleaning tools.

``ftfy`` and ``langdetect`` (used by the reference) are not part of this
image: ``fix_text`` uses ftfy when it is importable and otherwise only applies
Unicode NFC normalisation plus the most common mojibake repairs;
``is_english`` uses langdetect when importable and otherwise a stop-word
ratio test (>= 8 % of word tokens are frequent English function words).
"""
import re
import unicodedata

try:
    import ftfy as _ftfy
except ImportError:
    _ftfy = None
try:
    from langdetect import detect as _detect
except ImportError:
    _detect = None

_MOJIBAKE = {"â€™": "’", "â€œ": "“",
             "â€\u009d": "”", "â€“": "–",
             "â€”": "—", "Ã©": "é", "Â ": " "}
_STOP = frozenset("the of and to a in is that it for was on with as be by at this are from "
                  "or an have not but had his they which you he were has her their all "
                  "been one we there can will would more if so about what when who".split())
_WORD = re.compile(r"[A-Za-zÀ-ɏ']+|[^\sA-Za-z]+")


def fix_text(text):
    if _ftfy is not None:
        return _ftfy.fix_text(text)
    for bad, good in _MOJIBAKE.items():
        text = text.replace(bad, good)
    return unicodedata.normalize("NFC", text)


def is_english(text):
    if _detect is not None:
        return _detect(text) == "en"
    words = _WORD.findall(text.lower())
    return bool(words) and sum(w in _STOP for w in words) >= 0.08 * len(words)
