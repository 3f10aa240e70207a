"""REST front-end for generation (reference ``megatron/text_generation_server.py``).

``PUT /api`` with the reference's JSON contract (``prompts`` (<= 128),
``tokens_to_generate``, ``logprobs``, ``temperature``, ``top_k``, ``top_p``,
``top_p_decay``, ``top_p_bound``, ``add_BOS``, ``stop_on_double_eol``,
``stop_on_eol``, ``prevent_newline_after_colon``, ``random_seed``, ``no_log``,
``beam_width``, ``stop_token``, ``length_penalty``) answering
``{"text", "segments", "logprobs"}`` or ``{"text", "segments", "scores"}``.

The app is FastAPI/uvicorn (the reference used Flask-RESTful; FastAPI gives
request validation and an ASGI server with the same ``PUT /api`` contract);
``GET /`` serves the small web UI in ``static/index.html`` (reference
``megatron/static``).  Validation
lives in :func:`parse_request` (pure, unit-tested); invalid requests get HTTP
400 with the reference's message (the reference answered some of them with
200).  Rank 0 serves; before each request it broadcasts a command code
(0 = generate, 1 = beam search) so the other ranks, parked in
:func:`worker_loop`, join the same collective generation call.
"""
import datetime
import json
import os
import threading

import torch
import torch.distributed as dist

from .api import beam_search_and_post_process, generate_and_post_process
from .communication import device

GENERATE_NUM = 0
BEAM_NUM = 1
STOP_NUM = 2
_lock = threading.Lock()


class RequestError(ValueError):
    pass


def _is_num(x):
    return type(x) in (int, float)


def parse_request(body):
    """Validate a request body -> ("generate" | "beam", kwargs, no_log)."""
    if not isinstance(body, dict) or "prompts" not in body:
        raise RequestError("prompts argument required")
    if "max_len" in body:
        raise RequestError("max_len is no longer used.  Replace with tokens_to_generate")
    if "sentences" in body:
        raise RequestError("sentences is no longer used.  Replace with prompts")
    prompts = body["prompts"]
    if not isinstance(prompts, list) or not all(isinstance(p, str) for p in prompts):
        raise RequestError("prompts is not a list of strings")
    if not prompts:
        raise RequestError("prompts is empty")
    if len(prompts) > 128:
        raise RequestError("Maximum number of prompts is 128")
    g = body.get
    n = g("tokens_to_generate", 64)
    if type(n) is not int or n < 0:
        raise RequestError("tokens_to_generate must be an integer greater than or equal to 0")
    logprobs = g("logprobs", False)
    if not isinstance(logprobs, bool):
        raise RequestError("logprobs must be a boolean value")
    if n == 0 and not logprobs:
        raise RequestError("tokens_to_generate=0 implies logprobs should be True")
    temperature = g("temperature", 1.0)
    if not _is_num(temperature) or not 0.0 < temperature <= 100.0:
        raise RequestError("temperature must be a positive number less than or equal to 100.0")
    top_k = g("top_k", 0)
    if type(top_k) is not int or not 0 <= top_k <= 1000:
        raise RequestError("top_k must be an integer equal to or greater than 0 and less than "
                           "or equal to 1000")
    top_p = g("top_p", 0.0)
    if "top_p" in body:
        if type(top_p) is not float:
            raise RequestError("top_p must be a positive float less than or equal to 1.0")
        if top_p > 0.0 and top_k > 0:
            raise RequestError("cannot set both top-k and top-p samplings.")
        if not 0 <= top_p <= 1.0:
            raise RequestError("top_p must be less than or equal to 1.0")
    top_p_decay = g("top_p_decay", 0.0)
    if "top_p_decay" in body:
        if type(top_p_decay) is not float:
            raise RequestError("top_p_decay must be a positive float less than or equal to 1.0")
        if top_p == 0.0:
            raise RequestError("top_p_decay cannot be set without top_p")
        if not 0 <= top_p_decay <= 1.0:
            raise RequestError("top_p_decay must be less than or equal to 1.0")
    top_p_bound = g("top_p_bound", 0.0)
    if "top_p_bound" in body:
        if type(top_p_bound) is not float:
            raise RequestError("top_p_bound must be a positive float less than or equal to top_p")
        if top_p == 0.0:
            raise RequestError("top_p_bound cannot be set without top_p")
        if not 0.0 < top_p_bound <= top_p:
            raise RequestError("top_p_bound must be greater than 0 and less than top_p")
    flags = {}
    for name in ("add_BOS", "stop_on_double_eol", "stop_on_eol",
                 "prevent_newline_after_colon", "no_log"):
        flags[name] = g(name, False)
        if not isinstance(flags[name], bool):
            raise RequestError(f"{name} must be a boolean value")
    if any(len(p) == 0 for p in prompts) and not flags["add_BOS"]:
        raise RequestError("Empty prompts require add_BOS=true")
    random_seed = g("random_seed", -1)
    if "random_seed" in body and (type(random_seed) is not int or random_seed < 0):
        raise RequestError("random_seed must be a positive integer")
    beam_width = g("beam_width", None)
    if beam_width is not None:
        if type(beam_width) is not int or beam_width < 1:
            raise RequestError("beam_width must be an integer > 1")
        if len(prompts) > 1:
            raise RequestError("When doing beam_search, batch size must be 1")
    stop_token = g("stop_token", 50256)
    if type(stop_token) is not int:
        raise RequestError("stop_token must be an integer")
    length_penalty = g("length_penalty", 1)
    if "length_penalty" in body and type(length_penalty) is not float:
        raise RequestError("length_penalty must be a float")
    if beam_width is not None:
        return "beam", dict(prompts=prompts, tokens_to_generate=n, beam_size=beam_width,
                            add_BOS=flags["add_BOS"], stop_token=stop_token,
                            num_return_gen=beam_width, length_penalty=length_penalty,
                            prevent_newline_after_colon=flags["prevent_newline_after_colon"]), \
            flags["no_log"]
    return "generate", dict(prompts=prompts, tokens_to_generate=n,
                            return_output_log_probs=logprobs, top_k_sampling=top_k,
                            top_p_sampling=top_p, top_p_decay=top_p_decay,
                            top_p_bound=top_p_bound, temperature=temperature,
                            add_BOS=flags["add_BOS"], use_eod_token_for_early_termination=True,
                            stop_on_double_eol=flags["stop_on_double_eol"],
                            stop_on_eol=flags["stop_on_eol"],
                            prevent_newline_after_colon=flags["prevent_newline_after_colon"],
                            random_seed=random_seed), flags["no_log"]


def _send_choice(code):
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.broadcast(torch.tensor([code], dtype=torch.int64, device=device()), 0)


def handle(model, body, remote=None):
    """Run one validated request on rank 0 -> JSON-able dict (raises RequestError)."""
    kind, kwargs, no_log = parse_request(body)
    with _lock:
        if not no_log:
            print(f"request IP: {remote}\n{json.dumps(body)}\nstart time: "
                  f"{datetime.datetime.now()}", flush=True)
        try:
            if kind == "beam":
                _send_choice(BEAM_NUM)
                text, seg, scores = beam_search_and_post_process(model, **kwargs)
                return {"text": text, "segments": seg, "scores": scores}
            _send_choice(GENERATE_NUM)
            text, seg, logprobs, _ = generate_and_post_process(model, **kwargs)
            return {"text": text, "segments": seg, "logprobs": logprobs}
        except ValueError as e:
            raise RequestError(e.args[0]) from e


def worker_loop(model):
    """Non-serving ranks: follow rank 0's command codes until STOP_NUM."""
    while True:
        choice = torch.empty(1, dtype=torch.int64, device=device())
        dist.broadcast(choice, 0)
        code = int(choice.item())
        try:
            if code == GENERATE_NUM:
                generate_and_post_process(model)
            elif code == BEAM_NUM:
                beam_search_and_post_process(model)
            elif code == STOP_NUM:
                return
        except ValueError:
            pass


def stop_workers():
    _send_choice(STOP_NUM)


_INDEX_HTML = os.path.join(os.path.dirname(os.path.abspath(__file__)), "static", "index.html")


class MegatronServer:

    def __init__(self, model):
        from fastapi import FastAPI, Request
        from fastapi.responses import JSONResponse, PlainTextResponse
        self.app = FastAPI()
        self.model = model

        @self.app.get("/")
        def index():
            from fastapi.responses import HTMLResponse
            with open(_INDEX_HTML, encoding="utf-8") as f:
                return HTMLResponse(f.read())

        @self.app.put("/api")
        def api(body: dict, request: Request):  # sync handler -> worker thread
            try:
                return JSONResponse(handle(self.model, body, request.client.host
                                           if request.client else None))
            except RequestError as e:
                return PlainTextResponse(str(e.args[0]), status_code=400)

    def run(self, url="0.0.0.0", port=5000):
        import uvicorn
        uvicorn.run(self.app, host=url, port=port, log_level="warning")
