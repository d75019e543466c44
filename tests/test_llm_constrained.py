"""CPU tests of llama-server's request contract beyond plain sampling (VERDICT r5 "Next round" 5):
GBNF grammars, JSON mode / JSON schema (models/llm/grammar.py), ``n_probs`` and OpenAI
``logprobs``, HTTP 400 for fields the server cannot honour; and the scheduler's prompt-time
metrics."""
import json
import math
import time

import pytest
import torch

from k8s_nvidia_gpus_amd.models.llm import grammar as G
from k8s_nvidia_gpus_amd.models.llm import tiny


@pytest.fixture(scope="module")
def tiny_model(tmp_path_factory):
    from k8s_nvidia_gpus_amd.models.llm.synthetic import write_synthetic_gguf

    p = str(tmp_path_factory.mktemp("llm") / "tiny.gguf")
    write_synthetic_gguf(p, tiny())
    return p


def _load(path, slots=4, ctx=512):
    from k8s_nvidia_gpus_amd.models.llm.synthetic import load

    return load(path, device="cpu", max_ctx=ctx, slots=slots)


@pytest.fixture(scope="module")
def client(tiny_model):
    from fastapi.testclient import TestClient

    from k8s_nvidia_gpus_amd.models.llm.server import Scheduler, create_app

    eng, tok = _load(tiny_model)
    sched = Scheduler(eng, tok, parallel=4, ubatch=64)
    c = TestClient(create_app({"scheduler": sched, "tok": tok, "model": "tiny"}))
    c.sched = sched
    c.tok = tok
    yield c
    sched.close()


def _complete(m, text):
    st = m.feed(m.start, text.encode())
    return st is not None and G.Matcher.complete(st)


# ------------------------------------------------------------------------------ grammar unit tests
def test_json_object_grammar_accepts_json_and_rejects_the_rest():
    m = G.matcher_for(G.JSON_OBJECT_GBNF)
    for ok in ['{}', '{"a": 1}', '{"a": [1, -2.5e3, "x\\n\\u00e9", true, null, {"b": {}}]}',
               '{"é": "東京"}', '{ "a" : "b" }\n']:
        assert _complete(m, ok), ok
        json.loads(ok)
    for bad in ['[1]', '{"a":}', '{a: 1}', '{"a": 01}', '{"a": "\x01"}', '{} x', '"s"']:
        assert not _complete(m, bad), bad
    assert m.feed(m.start, b'{"a": [1, ') is not None          # a live prefix


def test_gbnf_features_and_errors():
    m = G.Matcher(G.parse_gbnf('root ::= ("ab" | [0-9]{2,3})+ "." # comment\n'))
    assert _complete(m, "ab.") and _complete(m, "12ab999.") and _complete(m, "1234.")
    assert not _complete(m, "1.") and not _complete(m, "abab")
    m = G.Matcher(G.parse_gbnf('root ::= [^x]* "x"\n'))
    assert _complete(m, "hello x") and not _complete(m, "xx")
    m = G.Matcher(G.parse_gbnf('root ::= item ("," item)?\nitem ::= "\\u00e9"+ | .\n'))
    assert _complete(m, "éé,?") and _complete(m, "z")
    for bad, what in [('root ::= foo', "never defined"), ('x ::= "a"', "no 'root'"),
                      ('root ::= root "a" | "b"', "left recursion"),
                      ('root ::= "a"\nroot ::= "b"', "defined twice"),
                      ('root ::= [a-', "unterminated"), ('root ::= "a" b ::= "c"', "newline")]:
        with pytest.raises(G.GrammarError, match=what):
            G.parse_gbnf(bad)


def test_json_schema_subset_and_unsupported_keywords():
    schema = {"type": "object",
              "properties": {"name": {"type": "string", "maxLength": 8}, "age": {"type": "integer"},
                             "tags": {"type": "array", "items": {"type": "string"}, "maxItems": 2},
                             "kind": {"enum": ["a", "b"]}},
              "required": ["name", "kind"]}
    m = G.matcher_for(G.json_schema_to_gbnf(schema))
    assert _complete(m, '{"name": "x", "kind": "a"}')
    assert _complete(m, '{"name": "x", "age": 3, "tags": ["p", "q"], "kind": "b"}')
    assert not _complete(m, '{"kind": "a"}')                          # required name missing
    assert not _complete(m, '{"name": "x", "tags": ["a", "b", "c"], "kind": "a"}')   # maxItems
    assert not _complete(m, '{"name": "x", "kind": "c"}')             # enum
    assert not _complete(m, '{"name": "123456789", "kind": "a"}')     # maxLength
    rec = {"$defs": {"node": {"type": "object", "properties": {
        "v": {"type": "integer"}, "kids": {"type": "array", "items": {"$ref": "#/$defs/node"}}},
        "required": ["v"]}}, "$ref": "#/$defs/node"}
    m = G.matcher_for(G.json_schema_to_gbnf(rec))
    assert _complete(m, '{"v": 1, "kids": [{"v": 2}, {"v": 3, "kids": []}]}')
    for bad, word in [({"type": "string", "pattern": "a+"}, "pattern"),
                      ({"type": "number", "minimum": 1}, "minimum"),
                      ({"$ref": "#/$defs/missing"}, "ref"), ({"type": "tuple"}, "tuple")]:
        with pytest.raises(G.GrammarError, match=word):
            G.json_schema_to_gbnf(bad)


def test_token_mask_follows_the_grammar(tiny_model):
    """The trie walk allows exactly the tokens whose bytes keep the text in the language; stop
    tokens only once the text is complete."""
    _, tok = _load(tiny_model)
    stop = tok.stop_ids()
    gs = G.GrammarState(G.matcher_for(G.JSON_OBJECT_GBNF), tok, stop)
    tb = tok.token_bytes()
    allowed = set(gs.allowed_ids())
    brute = {i for i, b in enumerate(tb) if b and gs.m.feed(gs.state, b) is not None}
    assert allowed == brute and tok.vocab["{"] in allowed and not set(stop) & allowed
    for piece in ["{", '"', "a", '"', ":", " ", "1", "}"]:
        tid = tok.vocab[piece] if piece != " " else tok.encode(" ")[0]
        assert gs.accepts(tid), piece
        gs.advance(tid)
    assert set(stop) <= set(gs.allowed_ids())
    mask = gs.mask(len(tb), "cpu")
    assert mask.dtype == torch.bool and bool(mask[stop[0]])


# ------------------------------------------------------------------------------ through the server
def test_json_schema_request_returns_schema_valid_json(client):
    schema = {"type": "object", "properties": {"ok": {"type": "boolean"},
                                               "n": {"type": "integer"}},
              "required": ["ok", "n"]}
    r = client.post("/completion", json={"prompt": "answer: ", "n_predict": 200, "temperature": 0,
                                         "json_schema": schema, "cache_prompt": False})
    assert r.status_code == 200, r.text
    out = json.loads(r.json()["content"])
    assert set(out) == {"ok", "n"} and isinstance(out["ok"], bool) and isinstance(out["n"], int)
    r = client.post("/v1/chat/completions", json={
        "messages": [{"role": "user", "content": "hi"}], "max_tokens": 200, "temperature": 0,
        "response_format": {"type": "json_schema",
                            "json_schema": {"name": "x", "schema": schema, "strict": True}}})
    assert r.status_code == 200, r.text
    out = json.loads(r.json()["choices"][0]["message"]["content"])
    assert set(out) == {"ok", "n"}


def test_json_object_mode_output_parses(client):
    """response_format json_object: the output is a JSON object (the biases only make the random
    model close its strings and objects quickly; the grammar does the rest)."""
    tok = client.tok
    bias = [[tok.vocab["}"], 6.0], [tok.vocab['"'], 3.0]]
    for seed in range(3):
        r = client.post("/v1/completions", json={
            "prompt": f"json {seed}: ", "max_tokens": 300, "temperature": 0.7, "seed": seed,
            "logit_bias": bias, "response_format": {"type": "json_object"}})
        assert r.status_code == 200, r.text
        text = r.json()["choices"][0]["text"]
        assert isinstance(json.loads(text), dict), text
        assert r.json()["choices"][0]["finish_reason"] == "stop"


def test_grammar_field_constrains_output(client):
    r = client.post("/completion", json={"prompt": "pick: ", "n_predict": 50, "temperature": 0,
                                         "grammar": 'root ::= ("yes" | "no") "!"\n'})
    assert r.status_code == 200, r.text
    assert r.json()["content"] in ("yes!", "no!")


def test_n_probs_matches_softmax_of_the_logits(client, tiny_model):
    eng, tok = _load(tiny_model)
    ids = tok.encode("hello world")
    ref = torch.log_softmax(eng.prefill(ids, 0).float(), -1)
    want = torch.topk(ref, 5)
    r = client.post("/completion", json={"prompt": ids, "n_predict": 3, "temperature": 0,
                                         "n_probs": 5, "cache_prompt": False})
    assert r.status_code == 200, r.text
    probs = r.json()["completion_probabilities"]
    assert len(probs) == 3
    first = probs[0]
    assert [t["id"] for t in first["top_logprobs"]] == want.indices.tolist()
    for t, v in zip(first["top_logprobs"], want.values.tolist()):
        assert t["logprob"] == pytest.approx(v, abs=1e-4)
    assert first["id"] == want.indices[0].item()                     # greedy picked the top one
    assert first["logprob"] == pytest.approx(want.values[0].item(), abs=1e-4)
    assert isinstance(first["bytes"], list) and isinstance(first["token"], str)
    # post-sampling probabilities of a greedy draw: the chosen token has probability 1
    r = client.post("/completion", json={"prompt": ids, "n_predict": 1, "temperature": 0,
                                         "n_probs": 3, "post_sampling_probs": True})
    p = r.json()["completion_probabilities"][0]
    assert p["prob"] == 1.0 and p["top_probs"][0]["id"] == p["id"]


def test_openai_logprobs_shapes(client):
    r = client.post("/v1/chat/completions", json={
        "messages": [{"role": "user", "content": "hi"}], "max_tokens": 4, "temperature": 0,
        "logprobs": True, "top_logprobs": 3})
    assert r.status_code == 200, r.text
    lp = r.json()["choices"][0]["logprobs"]["content"]
    assert 1 <= len(lp) <= 4 and all(len(e["top_logprobs"]) == 3 for e in lp)
    assert all(e["logprob"] <= 0 for e in lp)
    r = client.post("/v1/completions", json={"prompt": "hello", "max_tokens": 4, "temperature": 0,
                                             "logprobs": 2})
    lp = r.json()["choices"][0]["logprobs"]
    assert len(lp["tokens"]) == len(lp["token_logprobs"]) == len(lp["top_logprobs"]) >= 1
    assert all(len(d) <= 2 for d in lp["top_logprobs"]) and lp["text_offset"][0] == 0
    # streamed: every chunk with text carries its tokens' entries
    with client.stream("POST", "/v1/chat/completions", json={
            "messages": [{"role": "user", "content": "hi"}], "max_tokens": 5, "temperature": 0,
            "logprobs": True, "stream": True, "ignore_eos": True}) as s:
        chunks = [json.loads(line[6:]) for line in s.iter_lines()
                  if line.startswith("data: {")]
    n = sum(len(c["choices"][0].get("logprobs", {}).get("content", [])) for c in chunks
            if c["choices"][0].get("logprobs"))
    assert n == 5


@pytest.mark.parametrize("extra,word", [
    ({"n": 2}, "n"),
    ({"response_format": {"type": "xml"}}, "response_format"),
    ({"json_schema": {"type": "string", "pattern": "x"}}, "pattern"),
    ({"grammar": "root ::= missing"}, "missing"),
    ({"grammar": 'root ::= "a"', "json_schema": {"type": "object"}}, "only one"),
    ({"n_probs": -1}, "n_probs"),
])
def test_unsupported_fields_are_400_not_silently_ignored(client, extra, word):
    r = client.post("/completion", json=dict({"prompt": "x", "n_predict": 2}, **extra))
    assert r.status_code == 400, r.text
    assert word in r.json()["detail"]


def test_chat_top_logprobs_without_logprobs_is_400(client):
    r = client.post("/v1/chat/completions", json={"messages": [{"role": "user", "content": "x"}],
                                                  "top_logprobs": 2})
    assert r.status_code == 400 and "logprobs" in r.json()["detail"]


# ------------------------------------------------------------------------------ metrics
class SlowBatchEngine:
    """prefill_many takes 0.2 s however many prompts it gets."""

    def __init__(self, eng):
        self.e = eng
        self.slots, self.max_ctx, self.cfg, self.gpu = eng.slots, eng.max_ctx, eng.cfg, False
        self.device = eng.device
        self.calls = 0

    def prefill_many(self, items):
        self.calls += 1
        time.sleep(0.2)
        return [self.e.prefill(t, s, st) for t, s, st in items]

    def prefill(self, ids, slot, start=0):
        return self.e.prefill(ids, slot, start)

    def decode(self, *a):
        return self.e.decode(*a)


def _wait(job, timeout=60):
    t0 = time.time()
    while True:
        kind, val = job.out.get(timeout=max(0.1, timeout - (time.time() - t0)))
        if kind == "done":
            return val
        assert kind != "error", val


def test_batched_prompts_add_one_batch_time_to_prefill_seconds(tiny_model):
    from k8s_nvidia_gpus_amd.models.llm import server as S

    eng, tok = _load(tiny_model)
    slow = SlowBatchEngine(eng)
    sched = S.Scheduler(slow, tok, parallel=3, ubatch=64, autostart=False)
    try:
        jobs = [sched.submit(S.Job(ids=tok.encode(t), max_new=1, ignore_eos=True))
                for t in ("a cozy cabin", "hello world", "the lazy dog")]
        sched.start()
        for j in jobs:
            _wait(j)
    finally:
        sched.close()
    m = sched.metrics
    assert slow.calls == 1 and m["prefill_batches_total"] == 1
    assert m["prefill_chunks_total"] == 3
    assert 0.2 <= m["prefill_seconds_total"] < 0.5, m         # once, not 3 x 0.2
    shares = [j.t_prefill for j in jobs]
    # token shares of that one batch time (so each below it, and summing to it)
    assert all(s < m["prefill_seconds_total"] for s in shares)
    assert sum(shares) == pytest.approx(m["prefill_seconds_total"], rel=1e-6)


def test_no_prompt_batch_prefills_each_prompt_alone(tiny_model):
    from k8s_nvidia_gpus_amd.models.llm import server as S

    eng, tok = _load(tiny_model)
    slow = SlowBatchEngine(eng)
    sched = S.Scheduler(slow, tok, parallel=3, ubatch=64, autostart=False, prompt_batch=False)
    try:
        jobs = [sched.submit(S.Job(ids=tok.encode(t), max_new=1, ignore_eos=True))
                for t in ("a cozy cabin", "hello world")]
        sched.start()
        for j in jobs:
            _wait(j)
    finally:
        sched.close()
    assert slow.calls == 0 and sched.metrics["prefill_chunks_total"] == 2
