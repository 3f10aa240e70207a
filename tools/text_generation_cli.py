"""Interactive client for the REST server (reference ``tools/text_generation_cli.py``,
which was Python-2 ``urllib2``; this one is Python 3 stdlib only).

    python tools/text_generation_cli.py http://HOST:5000/api
"""
import json
import sys
import urllib.request


def put(url, payload):
    req = urllib.request.Request(url, data=json.dumps(payload).encode(), method="PUT",
                                 headers={"Content-Type": "application/json"})
    with urllib.request.urlopen(req) as resp:
        return json.load(resp)


if __name__ == "__main__":
    url = sys.argv[1]
    while True:
        sentence = input("Enter prompt: ")
        n = int(input("Enter number of tokens to generate: "))
        out = put(url, {"prompts": [sentence], "tokens_to_generate": n})
        print("Megatron Response: ")
        print(out["text"][0])
