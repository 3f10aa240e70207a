"""Filter a list of urls (reference ``tools/openwebtext/blacklist_urls.py``).

    python blacklist_urls.py <dir with *.txt url lists> <clean_urls.txt> [--domain_blacklist FILE]

Drops urls whose registered domain is blacklisted (media / file hosts and
social sites that yield no article text), whose path ends in a binary or
media extension, that are <= 8 characters, malformed, or duplicates.  The
registered domain is the label before the public suffix (a built-in list of
two-level suffixes replaces the ``tldextract`` package).
"""
import argparse
import glob
import os
import re
from urllib.parse import urlsplit

DOMAIN_BLACKLIST = frozenset("""
500px aapks akamaihd amazon apple artstation bandcamp bbc behance bit bitly blogspot
dailymotion deviantart discord dropbox ebay facebook fbcdn flickr giphy github gfycat
google googleusercontent gyazo imgur instagram itunes kickstarter linkedin liveleak
mediafire mega microsoft myspace netflix pastebin patreon photobucket pinterest
prntscr puu quora reddit redd redditmedia scribd soundcloud spotify steampowered
streamable t tinypic tumblr twimg twitch twitter vimeo vine wikimedia wordpress
youtu youtube
""".split())
EXT_BLACKLIST = tuple(
    ".3gp .7z .ai .aif .apk .app .avi .bin .bmp .bz2 .css .csv .dat .deb .dmg .doc .docx "
    ".exe .gif .gifv .gz .iso .jar .jpeg .jpg .js .log .mid .midi .mkv .mov .mp3 .mp4 .mpeg "
    ".mpg .ogg .ogv .otf .pdf .pkg .png .pps .ppt .pptx .psd .py .qt .ram .rar .sql .svg "
    ".swf .tar.gz .tar .tgz .tiff .ttf .txt .wav .webm .wma .wmv .xls .xlsx .xml .xz .zip".split())
_TWO_LEVEL = frozenset("co.uk org.uk ac.uk gov.uk com.au net.au org.au co.jp co.nz co.in "
                       "com.br com.cn com.mx co.za com.tr com.sg".split())
URL_RE = re.compile(
    r"^https?://(?:(?:[A-Z0-9](?:[A-Z0-9-]{0,61}[A-Z0-9])?\.)+(?:[A-Z]{2,6}\.?|[A-Z0-9-]{2,}\.?)"
    r"|\d{1,3}\.\d{1,3}\.\d{1,3}\.\d{1,3})(?::\d+)?(?:/?|[/?]\S+)$", re.IGNORECASE)


def registered_domain(url):
    host = (urlsplit(url).hostname or "").lower().rstrip(".")
    labels = host.split(".")
    if len(labels) >= 3 and ".".join(labels[-2:]) in _TWO_LEVEL:
        return labels[-3]
    return labels[-2] if len(labels) >= 2 else host


def classify(url, seen, blacklist=DOMAIN_BLACKLIST):
    try:
        if registered_domain(url) in blacklist:
            return "domain"
    except ValueError:
        return "malformed"
    if url.split("?")[0].lower().endswith(EXT_BLACKLIST):
        return "extension"
    if len(url) <= 8:
        return "short"
    if URL_RE.match(url) is None:
        return "malformed"
    if url in seen:
        return "duplicate"
    return None


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("path")
    p.add_argument("output")
    p.add_argument("--domain_blacklist", default=None, help="file with one domain label per line")
    a = p.parse_args(argv)
    blacklist = DOMAIN_BLACKLIST
    if a.domain_blacklist:
        with open(a.domain_blacklist) as f:
            blacklist = blacklist | {x.strip() for x in f if x.strip()}
    seen, counts = [], {}
    seen_set = set()
    for fname in sorted(glob.glob(os.path.join(a.path, "*.txt"))):
        with open(fname) as f:
            for line in f:
                url = line.strip()
                why = classify(url, seen_set, blacklist)
                counts[why or "kept"] = counts.get(why or "kept", 0) + 1
                if why is None:
                    seen_set.add(url)
                    seen.append(url)
    with open(a.output, "w") as f:
        for url in seen:
            f.write(url + "\n")
    print(counts)
    return counts


if __name__ == "__main__":
    main()
