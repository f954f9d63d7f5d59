"""InferenceService predictor HTTP server (KServe protocol surface) over :class:`Engine`.

Endpoints (KServe v1 / Open Inference Protocol v2 / OpenAI-style completions):

* ``GET /``, ``GET /v1/models``, ``GET /v1/models/<name>`` (``{"name", "ready"}``),
  ``GET /v2/health/live``, ``/v2/health/ready``, ``GET /v2/models/<name>[/ready]``
* ``POST /v1/models/<name>:predict`` ``{"instances": [{"prompt": str | "token_ids": [int],
  "max_new_tokens", "temperature", "top_p"}]}`` -> ``{"predictions": [...]}``
* ``POST /v2/models/<name>/infer`` with a ``BYTES`` ``text_input`` or ``INT64`` ``input_ids``
  tensor -> ``text_output`` / ``output_ids``
* ``POST /v1/completions`` ``{"prompt", "max_tokens", "temperature", "top_p"}``
* ``GET /metrics`` (prometheus: request count/latency, tokens generated, TTFT)

Text is tokenised with a HuggingFace ``tokenizer.json`` when ``--tokenizer`` points at one
(the ``tokenizers`` package is installed), else with a byte-level fallback (ids 0..255) so
the random-init benchmark model can be driven end to end without downloads.
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import threading
import time
from typing import List, Optional

from .engine import Request, Scheduler, build_engine

log = logging.getLogger("predictor")


class ByteTokenizer:
    def encode(self, text: str) -> List[int]:
        return list(text.encode("utf-8"))

    def decode(self, ids: List[int]) -> str:
        return bytes(i for i in ids if 0 <= i < 256).decode("utf-8", errors="replace")


class HFTokenizer:
    def __init__(self, path: str):
        from tokenizers import Tokenizer
        self.t = Tokenizer.from_file(path)

    def encode(self, text):
        return self.t.encode(text).ids

    def decode(self, ids):
        return self.t.decode(ids)


def create_app(sched: Scheduler, model_name: str, tokenizer=None, registry=None):
    from flask import Flask, Response, jsonify, request
    from prometheus_client import CollectorRegistry, Counter, Histogram, generate_latest, CONTENT_TYPE_LATEST

    tok = tokenizer or ByteTokenizer()
    reg = registry or CollectorRegistry()
    m_req = Counter("predictor_requests_total", "inference requests", ["endpoint", "status"], registry=reg)
    m_lat = Histogram("predictor_request_seconds", "request latency", ["endpoint"], registry=reg)
    m_ttft = Histogram("predictor_ttft_seconds", "time to first token", registry=reg)
    m_tok = Counter("predictor_generated_tokens_total", "generated tokens", registry=reg)
    app = Flask("predictor")

    def run(prompts: List[List[int]], max_new, temperature, top_p, timeout=600.0):
        reqs = [sched.submit(Request(prompt=p, max_new_tokens=max_new, temperature=temperature, top_p=top_p))
                for p in prompts]
        for r in reqs:
            if not r.done.wait(timeout):
                raise TimeoutError("generation timed out")
            if r.error:
                raise ValueError(r.error)
            m_ttft.observe(max(0.0, r.t_first - r.t_submit))
            m_tok.inc(len(r.output))
        return reqs

    def parse_instance(inst):
        if isinstance(inst, str):
            return tok.encode(inst), {}
        ids = inst.get("token_ids") or tok.encode(inst.get("prompt", inst.get("text", "")))
        return ids, inst

    @app.get("/")
    def root():
        return jsonify({"status": "alive"})

    @app.get("/v2/health/live")
    def live():
        return jsonify({"live": True})

    @app.get("/v2/health/ready")
    def ready():
        # a poisoned tensor-parallel communicator (one-shot all-reduce timeout) makes the
        # predictor unready so the InferenceService pod is taken out of rotation / restarted
        ok = getattr(sched.e, "healthy", True)
        return jsonify({"ready": ok}), (200 if ok else 503)

    @app.get("/v1/models")
    def models():
        return jsonify({"models": [model_name]})

    @app.get("/v1/models/<name>")
    def model_status(name):
        if name != model_name:
            return jsonify({"error": f"model {name} not found"}), 404
        return jsonify({"name": name, "ready": True})

    @app.get("/v2/models/<name>")
    @app.get("/v2/models/<name>/ready")
    def model_meta(name):
        if name != model_name:
            return jsonify({"error": f"model {name} not found"}), 404
        return jsonify({"name": name, "ready": True, "platform": "kfamd-mi355x",
                        "inputs": [{"name": "text_input", "datatype": "BYTES", "shape": [-1]},
                                   {"name": "input_ids", "datatype": "INT64", "shape": [-1]}],
                        "outputs": [{"name": "text_output", "datatype": "BYTES", "shape": [-1]}]})

    @app.post("/v1/models/<name>:predict")
    def predict(name):
        t0 = time.time()
        if name != model_name:
            m_req.labels("v1", "404").inc()
            return jsonify({"error": f"model {name} not found"}), 404
        body = request.get_json(force=True, silent=True) or {}
        insts = body.get("instances") or []
        try:
            parsed = [parse_instance(i) for i in insts]
            out = []
            for ids, opts in parsed:
                r = run([ids], int(opts.get("max_new_tokens", body.get("max_new_tokens", 32))),
                        float(opts.get("temperature", 0.0)), float(opts.get("top_p", 1.0)))[0]
                out.append({"token_ids": r.output, "text": tok.decode(r.output)})
        except (ValueError, TimeoutError) as e:
            m_req.labels("v1", "400").inc()
            return jsonify({"error": str(e)}), 400
        m_req.labels("v1", "200").inc()
        m_lat.labels("v1").observe(time.time() - t0)
        return jsonify({"predictions": out})

    @app.post("/v2/models/<name>/infer")
    def infer(name):
        t0 = time.time()
        if name != model_name:
            return jsonify({"error": f"model {name} not found"}), 404
        body = request.get_json(force=True, silent=True) or {}
        params = body.get("parameters") or {}
        prompts, as_text = [], True
        for inp in body.get("inputs") or []:
            if inp.get("name") == "input_ids":
                prompts.append([int(x) for x in inp.get("data", [])])
                as_text = False
            elif inp.get("name") == "text_input":
                prompts += [tok.encode(s) for s in inp.get("data", [])]
        if not prompts:
            return jsonify({"error": "no text_input or input_ids tensor"}), 400
        try:
            reqs = run(prompts, int(params.get("max_new_tokens", 32)), float(params.get("temperature", 0.0)),
                       float(params.get("top_p", 1.0)))
        except (ValueError, TimeoutError) as e:
            return jsonify({"error": str(e)}), 400
        m_req.labels("v2", "200").inc()
        m_lat.labels("v2").observe(time.time() - t0)
        if as_text:
            outs = [{"name": "text_output", "datatype": "BYTES", "shape": [len(reqs)],
                     "data": [tok.decode(r.output) for r in reqs]}]
        else:
            outs = [{"name": "output_ids", "datatype": "INT64", "shape": [len(reqs), len(reqs[0].output)],
                     "data": [t for r in reqs for t in r.output]}]
        return jsonify({"model_name": model_name, "id": body.get("id", ""), "outputs": outs})

    @app.post("/v1/completions")
    def completions():
        body = request.get_json(force=True, silent=True) or {}
        prompt = body.get("prompt", "")
        prompts = prompt if isinstance(prompt, list) else [prompt]
        try:
            reqs = run([p if isinstance(p, list) else tok.encode(p) for p in prompts], int(body.get("max_tokens", 16)),
                       float(body.get("temperature", 0.0)), float(body.get("top_p", 1.0)))
        except (ValueError, TimeoutError) as e:
            return jsonify({"error": {"message": str(e)}}), 400
        return jsonify({"object": "text_completion", "model": model_name, "created": int(time.time()),
                        "choices": [{"index": i, "text": tok.decode(r.output), "token_ids": r.output,
                                     "finish_reason": "length"} for i, r in enumerate(reqs)],
                        "usage": {"prompt_tokens": sum(len(r.prompt) for r in reqs),
                                  "completion_tokens": sum(len(r.output) for r in reqs)}})

    @app.get("/metrics")
    def metrics():
        return Response(generate_latest(reg), content_type=CONTENT_TYPE_LATEST)

    return app


def main(argv=None):
    p = argparse.ArgumentParser(description="kfamd InferenceService predictor")
    p.add_argument("--model-name", default=os.environ.get("MODEL_NAME", "llama3-8b"))
    p.add_argument("--model", default=os.environ.get("KFAMD_MODEL", "llama3-8b"), help="architecture preset")
    p.add_argument("--checkpoint", default=os.environ.get("STORAGE_PATH"))
    p.add_argument("--tokenizer", default=None)
    p.add_argument("--port", type=int, default=int(os.environ.get("PORT", "8080")))
    p.add_argument("--host", default="0.0.0.0")
    p.add_argument("--slots", type=int, default=64)
    p.add_argument("--max-len", type=int, default=4096)
    p.add_argument("--layers", type=int, default=None)
    p.add_argument("--tp", type=int, default=int(os.environ.get("WORLD_SIZE", "1")),
                   help="tensor-parallel degree (one process per GPU under kfamd-launch; rank 0 serves HTTP)")
    a = p.parse_args(argv)
    logging.basicConfig(level=logging.INFO)
    st = None
    if a.tp > 1:
        import torch.distributed as dist

        from ..parallel.state import init_distributed
        from .tp import TPLeaderEngine, follower_loop
        st = init_distributed(tp=a.tp)
        ctrl = dist.new_group(backend="gloo")      # command channel (host objects)
    eng = build_engine(a.model, n_slots=a.slots, max_len=a.max_len, checkpoint=a.checkpoint, n_layers=a.layers,
                       st=st, device=None if st is None else str(st.device))
    if st is not None:
        if st.rank != 0:
            n = follower_loop(eng, ctrl)
            log.info("TP follower rank %d done after %d commands", st.rank, n)
            return
        eng = TPLeaderEngine(eng, ctrl)
    sched = Scheduler(eng, max_batch=a.slots).start()
    tok = HFTokenizer(a.tokenizer) if a.tokenizer else None
    app = create_app(sched, a.model_name, tok)
    from werkzeug.serving import make_server
    srv = make_server(a.host, a.port, app, threaded=True)
    log.info("predictor %s serving on %s:%d", a.model_name, a.host, a.port)
    srv.serve_forever()


if __name__ == "__main__":
    main()
