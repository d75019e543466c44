"""CPU tests of the in-tree Qwen2 LLM family: GGUF container, K-quant codecs (against independent
scalar decoders written from the format description), tokenizer / ChatML, the engine's reference
path (incremental decode == full prefill), and the llama-server-compatible API with continuous
batching (FastAPI TestClient, no GPU)."""
import json

import numpy as np
import pytest
import torch

from k8s_nvidia_gpus_amd.models.llm import gguf, quants, tiny
from k8s_nvidia_gpus_amd.models.llm.config import from_gguf, to_gguf_metadata, use_more_bits


# ----------------------------------------------------------------- scalar reference decoders
def _f16(b):
    return float(np.frombuffer(bytes(b), "<f2")[0])


def scalar_q4_k(block: bytes) -> list:
    d, dmin = _f16(block[0:2]), _f16(block[2:4])
    sc = block[4:16]
    qs = block[16:144]

    def scale_min(j):
        if j < 4:
            return sc[j] & 63, sc[j + 4] & 63
        return (sc[j + 4] & 0xF) | ((sc[j - 4] >> 6) << 4), (sc[j + 4] >> 4) | ((sc[j] >> 6) << 4)

    out = []
    for c in range(4):
        s0, m0 = scale_min(2 * c)
        s1, m1 = scale_min(2 * c + 1)
        out += [d * s0 * (qs[32 * c + l] & 0xF) - dmin * m0 for l in range(32)]
        out += [d * s1 * (qs[32 * c + l] >> 4) - dmin * m1 for l in range(32)]
    return out


def scalar_q6_k(block: bytes) -> list:
    ql, qh = block[0:128], block[128:192]
    sc = np.frombuffer(bytes(block[192:208]), np.int8)
    d = _f16(block[208:210])
    y = [0.0] * 256
    for n in range(2):
        for l in range(32):
            is_ = l // 16
            q1 = ((ql[64 * n + l] & 0xF) | (((qh[32 * n + l] >> 0) & 3) << 4)) - 32
            q2 = ((ql[64 * n + l + 32] & 0xF) | (((qh[32 * n + l] >> 2) & 3) << 4)) - 32
            q3 = ((ql[64 * n + l] >> 4) | (((qh[32 * n + l] >> 4) & 3) << 4)) - 32
            q4 = ((ql[64 * n + l + 32] >> 4) | (((qh[32 * n + l] >> 6) & 3) << 4)) - 32
            y[128 * n + l] = d * sc[8 * n + is_] * q1
            y[128 * n + l + 32] = d * sc[8 * n + is_ + 2] * q2
            y[128 * n + l + 64] = d * sc[8 * n + is_ + 4] * q3
            y[128 * n + l + 96] = d * sc[8 * n + is_ + 6] * q4
    return y


@pytest.mark.parametrize("t,scalar,bs", [(gguf.Q4_K, scalar_q4_k, 144),
                                          (gguf.Q6_K, scalar_q6_k, 210)])
def test_vectorised_decoders_match_scalar_on_random_bytes(t, scalar, bs):
    rng = np.random.default_rng(7)
    raw = rng.integers(0, 256, (3, 2 * bs), dtype=np.uint8)
    # sane f16 scales (random bytes can be inf/nan)
    for r in range(3):
        for b in range(2):
            off = b * bs + (0 if t == gguf.Q4_K else 208)
            vals = np.array([0.01, 0.003] if t == gguf.Q4_K else [0.02], np.float16)
            raw[r, off:off + vals.nbytes] = vals.view(np.uint8)
    v = quants.dequantize(raw, t)
    for r in range(3):
        for b in range(2):
            ref = scalar(raw[r, b * bs:(b + 1) * bs].tobytes())
            np.testing.assert_allclose(v[r, b * 256:(b + 1) * 256], ref, rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("t,tol", [(gguf.Q4_K, 0.09), (gguf.Q6_K, 0.02), (gguf.Q8_0, 0.01)])
def test_quantisers_round_trip(t, tol):
    rng = np.random.default_rng(1)
    w = rng.standard_normal((8, 512)).astype(np.float32)
    back = quants.dequantize(quants.quantize(w, t), t)
    rel = np.linalg.norm(back - w) / np.linalg.norm(w)
    assert rel < tol, rel


def test_gguf_write_read_round_trip(tmp_path):
    p = str(tmp_path / "x.gguf")
    w = quants.quant_q4_k(np.random.default_rng(0).standard_normal((4, 256)).astype(np.float32))
    md = {"general.architecture": "qwen2", "a.f": 1.5, "a.s": "héllo", "a.b": True,
          "a.arr": ["x", "y z"], "a.ints": np.array([1, -2, 3], np.int32), "a.neg": -7}
    gguf.write_gguf(p, md, [("w", (256, 4), gguf.Q4_K, w),
                            ("v", (5,), gguf.F32, np.arange(5, dtype=np.float32)),
                            ("h", (2, 3), gguf.F16, np.ones((3, 2), np.float16))])
    with gguf.GGUFFile(p) as g:
        assert g.version == 3
        assert g.metadata["a.s"] == "héllo" and g.metadata["a.b"] is True
        assert g.metadata["a.arr"] == ["x", "y z"] and g.metadata["a.neg"] == -7
        assert list(g.metadata["a.ints"]) == [1, -2, 3]
        assert abs(g.metadata["a.f"] - 1.5) < 1e-6
        assert np.array_equal(g.raw("w"), w)
        assert np.array_equal(g.tensor("v"), np.arange(5, dtype=np.float32))
        assert g.tensor("h").shape == (3, 2)
        assert g.data_offset % 32 == 0
        s = gguf.summary(g)
        assert s["types"] == {"Q4_K": 1, "F32": 1, "F16": 1}


def test_gguf_rejects_bad_files(tmp_path):
    p = tmp_path / "bad.gguf"
    p.write_bytes(b"NOPE" + b"\0" * 40)
    with pytest.raises(gguf.GGUFError):
        gguf.GGUFFile(str(p))
    good = str(tmp_path / "t.gguf")
    gguf.write_gguf(good, {"k": 1}, [("v", (64,), gguf.F32, np.zeros(64, np.float32))])
    data = open(good, "rb").read()
    (tmp_path / "trunc.gguf").write_bytes(data[:-100])
    with pytest.raises(gguf.GGUFError):
        gguf.GGUFFile(str(tmp_path / "trunc.gguf"))


def test_config_round_trip_and_q4km_layers():
    c = tiny(layers=3)
    assert from_gguf(dict(to_gguf_metadata(c), **{"tokenizer.ggml.tokens": ["a"] * c.vocab})) \
        .dim == c.dim
    from k8s_nvidia_gpus_amd.models.llm import QWEN25_7B

    assert QWEN25_7B.head_dim == 128 and QWEN25_7B.group == 7
    assert 7.0e9 < QWEN25_7B.params() < 8.0e9
    more = [i for i in range(28) if use_more_bits(i, 28)]
    assert more[:3] == [0, 1, 2] and 27 in more and len(more) == 14


@pytest.fixture(scope="module")
def tiny_model(tmp_path_factory):
    from k8s_nvidia_gpus_amd.models.llm.synthetic import load, write_synthetic_gguf

    p = str(tmp_path_factory.mktemp("llm") / "tiny.gguf")
    write_synthetic_gguf(p, tiny())
    return p


def test_tokenizer_round_trip_and_specials(tiny_model):
    from k8s_nvidia_gpus_amd.models.llm.tokenizer import Tokenizer, chatml

    with gguf.GGUFFile(tiny_model) as g:
        tok = Tokenizer.from_gguf(g.metadata)
    for s in ["hello world", "The quick brown fox!\n  indented\ttab", "naïve café 東京 🙂"]:
        assert tok.decode(tok.encode(s)) == s
    text = chatml([{"role": "user", "content": "hi"}])
    ids = tok.encode(text)
    assert ids.count(tok.token_id("<|im_start|>")) == 3        # system, user, assistant
    assert tok.token_id("<|im_end|>") in tok.stop_ids()
    assert text.endswith("<|im_start|>assistant\n")
    assert "You are Qwen" in text
    assert "You are Qwen" not in chatml([{"role": "system", "content": "x"},
                                         {"role": "user", "content": "y"}])


def test_engine_incremental_decode_equals_prefill(tiny_model):
    from k8s_nvidia_gpus_amd.models.llm.synthetic import load

    eng, tok = load(tiny_model, device="cpu", max_ctx=256)
    ids = tok.encode("a cozy cabin in the woods, hello world")
    full = eng.prefill(ids, slot=0)
    eng.prefill(ids[:5], slot=1)
    for i in range(5, len(ids)):
        last = eng.decode([ids[i]], [i], [1])[0]
    torch.testing.assert_close(full, last, rtol=1e-4, atol=1e-4)
    # batched decode across slots equals per-slot decode
    eng.prefill(ids[:3], slot=2)
    b = eng.decode([ids[-1], ids[3]], [len(ids), 3], [0, 2])
    eng2, _ = load(tiny_model, device="cpu", max_ctx=256)
    eng2.prefill(ids, 0)
    eng2.prefill(ids[:3], 2)
    torch.testing.assert_close(b[0], eng2.decode([ids[-1]], [len(ids)], [0])[0])
    torch.testing.assert_close(b[1], eng2.decode([ids[3]], [3], [2])[0])


def test_prefill_rejects_overflow(tiny_model):
    from k8s_nvidia_gpus_amd.models.llm.synthetic import load

    eng, _ = load(tiny_model, device="cpu", max_ctx=256)
    with pytest.raises(ValueError):
        eng.prefill(list(range(300)), 0)


def test_sampling_modes():
    from k8s_nvidia_gpus_amd.models.llm.engine import sample

    lg = torch.tensor([0.0, 5.0, 1.0, 4.9])
    assert sample(lg) == 1
    g = torch.Generator().manual_seed(0)
    draws = {sample(lg, 1.0, top_k=2, generator=g) for _ in range(50)}
    assert draws <= {1, 3} and len(draws) == 2
    g = torch.Generator().manual_seed(0)
    assert {sample(lg, 1.0, top_p=0.3, generator=g) for _ in range(20)} == {1}


def test_sampling_llama_server_parameters():
    """min_p / penalties / logit_bias with llama.cpp's semantics and chain order."""
    from k8s_nvidia_gpus_amd.models.llm.sampling import SamplingParams, parse_logit_bias, sample_token

    lg = torch.tensor([2.0, 5.0, -1.0, 4.9, 0.5])
    # repeat penalty divides positive / multiplies negative logits of recent tokens
    p = SamplingParams(temperature=0.0, repeat_penalty=2.0)
    assert sample_token(lg, p, history=[1]) == 3            # 5/2 < 4.9
    assert sample_token(lg, SamplingParams(repeat_penalty=3.0), history=[1, 3]) == 0  # 1.67, 1.63 < 2
    p = SamplingParams(temperature=0.0, repeat_penalty=2.0, repeat_last_n=1)
    assert sample_token(lg, p, history=[1, 3]) == 1         # only the last token counts
    # presence / frequency penalties
    p = SamplingParams(temperature=0.0, frequency_penalty=0.06)
    assert sample_token(lg, p, history=[1, 1]) == 3         # 5 - 0.12 < 4.9
    assert sample_token(lg, p, history=[1]) == 1            # 5 - 0.06 > 4.9
    p = SamplingParams(temperature=0.0, presence_penalty=0.2)
    assert sample_token(lg, p, history=[1, 1, 1]) == 3
    # logit bias: OpenAI dict, llama.cpp pairs, false bans
    assert parse_logit_bias({"3": 1}) == {3: 1.0}
    assert parse_logit_bias([[1, False], [4, -2]]) == {1: -float("inf"), 4: -2.0}
    with pytest.raises(ValueError):
        parse_logit_bias({"9": 1}, vocab=5)
    assert sample_token(lg, SamplingParams(logit_bias={1: -float("inf")})) == 3
    # min_p: relative to the most likely token, before temperature
    g = torch.Generator().manual_seed(0)
    p = SamplingParams(temperature=5.0, min_p=0.5)
    assert {sample_token(lg, p, generator=g) for _ in range(200)} == {1, 3}
    p = SamplingParams(temperature=5.0, min_p=0.0)
    assert len({sample_token(lg, p, generator=g) for _ in range(400)}) == 5
    d = SamplingParams.from_request({"temperature": 0.2, "min_p": 0.1, "repeat_penalty": 1.1})
    assert (d.temperature, d.top_k, d.min_p, d.repeat_penalty, d.repeat_last_n) == (0.2, 40, 0.1, 1.1, 64)
    assert SamplingParams(temperature=0.0).plain_greedy and not d.plain_greedy


# ----------------------------------------------------------------- server
@pytest.fixture(scope="module")
def client(tiny_model):
    from fastapi.testclient import TestClient

    from k8s_nvidia_gpus_amd.models.llm.server import Scheduler, create_app
    from k8s_nvidia_gpus_amd.models.llm.synthetic import load

    eng, tok = load(tiny_model, device="cpu", max_ctx=256, slots=4)
    state = {"scheduler": None, "tok": tok, "model": "tiny"}
    app = create_app(state)
    c = TestClient(app)
    assert c.get("/health").status_code == 503              # llama-server: 503 while loading
    state["scheduler"] = Scheduler(eng, tok, parallel=4)
    yield c, eng, tok, state
    state["scheduler"].close()


def test_server_health_models_tokenize(client):
    c, eng, tok, _ = client
    assert c.get("/health").json() == {"status": "ok"}
    assert c.get("/v1/models").json()["data"][0]["id"] == "tiny"
    ids = c.post("/tokenize", json={"content": "hello world"}).json()["tokens"]
    assert ids == tok.encode("hello world")
    assert c.post("/detokenize", json={"tokens": ids}).json()["content"] == "hello world"


def test_server_completion_greedy_matches_engine(client, tiny_model):
    from k8s_nvidia_gpus_amd.models.llm.engine import generate
    from k8s_nvidia_gpus_amd.models.llm.synthetic import load

    c, eng, tok, _ = client
    r = c.post("/completion", json={"prompt": "the quick brown", "n_predict": 6,
                                    "temperature": 0}).json()
    assert r["tokens_predicted"] <= 6 and r["tokens_evaluated"] == len(tok.encode("the quick brown"))
    assert set(r["timings"]) >= {"prompt_n", "predicted_n", "predicted_per_second"}
    ref, _ = load(tiny_model, device="cpu", max_ctx=256)      # the server's engine is busy
    out = generate(ref, tok.encode("the quick brown"), 6, eos=tok.stop_ids())["tokens"]
    assert r["content"] == tok.decode(out)


def test_server_openai_chat_and_stream(client):
    c, eng, tok, _ = client
    body = {"model": "x", "messages": [{"role": "user", "content": "hello"}], "max_tokens": 5,
            "temperature": 0}
    r = c.post("/v1/chat/completions", json=body).json()
    assert r["object"] == "chat.completion"
    assert r["choices"][0]["message"]["role"] == "assistant"
    assert r["usage"]["completion_tokens"] <= 5
    assert r["choices"][0]["finish_reason"] in ("stop", "length")
    with c.stream("POST", "/v1/chat/completions", json=dict(body, stream=True)) as s:
        lines = [ln for ln in s.iter_lines() if ln]
    assert lines[-1] == "data: [DONE]"
    chunks = [json.loads(ln[6:]) for ln in lines[:-1]]
    text = "".join(ch["choices"][0]["delta"].get("content", "") for ch in chunks)
    assert text == r["choices"][0]["message"]["content"]
    assert chunks[-1]["choices"][0]["finish_reason"] == r["choices"][0]["finish_reason"]
    r2 = c.post("/v1/completions", json={"prompt": "hello", "max_tokens": 3, "temperature": 0})
    assert r2.json()["object"] == "text_completion"


def test_server_stop_strings_and_errors(client):
    c, eng, tok, _ = client
    r = c.post("/completion", json={"prompt": "hello", "n_predict": 20, "temperature": 0}).json()
    if len(r["content"]) > 2:
        stop = r["content"][1:3]
        r2 = c.post("/completion", json={"prompt": "hello", "n_predict": 20, "temperature": 0,
                                         "stop": [stop]}).json()
        assert stop not in r2["content"] and r["content"].startswith(r2["content"])
    assert c.post("/completion", json={"prompt": "x " * 400, "n_predict": 4}).status_code == 400
    assert c.post("/v1/chat/completions", json={"messages": []}).status_code == 400


def test_server_concurrent_requests_are_batched(client):
    """8 concurrent greedy requests over 4 slots: every answer equals its sequential answer and
    the scheduler ran multi-sequence decode steps."""
    from concurrent.futures import ThreadPoolExecutor

    c, eng, tok, state = client
    prompts = [f"hello world {i}" for i in range(8)]
    seq = [c.post("/completion", json={"prompt": p, "n_predict": 8, "temperature": 0}).json()
           ["content"] for p in prompts]
    steps0 = state["scheduler"].metrics["decode_steps_total"]
    toks0 = state["scheduler"].metrics["tokens_predicted_total"]
    with ThreadPoolExecutor(8) as ex:
        par = list(ex.map(lambda p: c.post("/completion", json={
            "prompt": p, "n_predict": 8, "temperature": 0}).json()["content"], prompts))
    assert par == seq
    m = state["scheduler"].metrics
    assert m["tokens_predicted_total"] - toks0 > m["decode_steps_total"] - steps0  # T > 1 steps
    assert "llamacpp_amdk8s_tokens_predicted_total" in c.get("/metrics").text


def test_server_seeded_sampling_is_reproducible(client):
    c, *_ = client
    body = {"prompt": "a cozy cabin", "n_predict": 8, "temperature": 1.0, "seed": 42}
    a = c.post("/completion", json=body).json()["content"]
    b = c.post("/completion", json=body).json()["content"]
    assert a == b


def test_server_prefill_error_reaches_its_request_and_serving_continues(tiny_model):
    """a job whose prefill raises (before it is active) gets a 500, not a hung worker."""
    from fastapi.testclient import TestClient

    from k8s_nvidia_gpus_amd.models.llm.server import Scheduler, create_app
    from k8s_nvidia_gpus_amd.models.llm.synthetic import load

    eng, tok = load(tiny_model, device="cpu", max_ctx=256, slots=2)
    real = eng.prefill
    calls = {"n": 0}

    def flaky(ids, slot, start=0):
        calls["n"] += 1
        if calls["n"] == 1:
            raise RuntimeError("probabilities contain inf")
        return real(ids, slot, start)

    eng.prefill = flaky
    state = {"scheduler": Scheduler(eng, tok, parallel=2), "tok": tok, "model": "tiny"}
    c = TestClient(create_app(state, request_timeout=30))
    try:
        r = c.post("/completion", json={"prompt": "hello", "n_predict": 3, "temperature": 0})
        assert r.status_code == 500 and "inf" in r.text
        ok = c.post("/completion", json={"prompt": "hello", "n_predict": 3, "temperature": 0})
        assert ok.status_code == 200 and ok.json()["tokens_predicted"] >= 1
        assert state["scheduler"].metrics["requests_failed_total"] == 1
    finally:
        state["scheduler"].close()


def test_server_cancels_abandoned_requests_and_times_out(tiny_model):
    """a stream the client closes is cancelled (its slot is freed before n_predict) and a
    blocking request never waits past the timeout."""
    import time as _t

    from fastapi.testclient import TestClient

    from k8s_nvidia_gpus_amd.models.llm import server as S
    from k8s_nvidia_gpus_amd.models.llm.synthetic import load

    eng, tok = load(tiny_model, device="cpu", max_ctx=256, slots=1)
    real_decode = eng.decode

    def slow_decode(*a, **k):
        _t.sleep(0.02)
        return real_decode(*a, **k)

    eng.decode = slow_decode
    sched = S.Scheduler(eng, tok, parallel=1)
    state = {"scheduler": sched, "tok": tok, "model": "tiny"}
    try:
        job = sched.submit(S.Job(ids=tok.encode("hello"), max_new=200))

        async def first_then_close():
            agen = S._astream(job, timeout=30)
            await agen.__anext__()                 # first token arrived: job is decoding
            await agen.aclose()                    # client went away

        import asyncio

        asyncio.run(first_then_close())
        assert job.cancelled
        t0 = _t.time()
        while sched.active and _t.time() - t0 < 5:
            _t.sleep(0.01)
        assert not sched.active and len(job.gen) < 200
        # blocking request with a short timeout: 504, and the job is cancelled
        c = TestClient(S.create_app(state, request_timeout=0.3))
        r = c.post("/completion", json={"prompt": "hello", "n_predict": 200, "temperature": 0})
        assert r.status_code == 504
        t0 = _t.time()
        while sched.active and _t.time() - t0 < 5:
            _t.sleep(0.01)
        assert not sched.active
    finally:
        sched.close()


def test_server_prompt_cache_reuses_slot_prefix(tiny_model):
    """cache_prompt: a follow-up prompt that extends a finished conversation goes to that
    conversation's slot and prefills only the new tokens; the answer equals the uncached one."""
    from fastapi.testclient import TestClient

    from k8s_nvidia_gpus_amd.models.llm.server import Scheduler, create_app
    from k8s_nvidia_gpus_amd.models.llm.synthetic import load

    eng, tok = load(tiny_model, device="cpu", max_ctx=256, slots=3)
    prefills = []
    real = eng.prefill

    def spy(ids, slot, start=0):
        prefills.append((len(ids), slot, start))
        return real(ids, slot, start)

    eng.prefill = spy
    sched = Scheduler(eng, tok, parallel=3)
    c = TestClient(create_app({"scheduler": sched, "tok": tok, "model": "tiny"}))
    try:
        c.post("/completion", json={"prompt": "other conversation", "n_predict": 2, "temperature": 0})
        first = c.post("/completion", json={"prompt": "the quick brown fox", "n_predict": 4,
                                            "temperature": 0}).json()
        assert first["timings"]["cache_n"] == 0
        slot_a = prefills[-1][1]
        follow = "the quick brown fox" + first["content"] + " jumps over"
        r = c.post("/completion", json={"prompt": follow, "n_predict": 5, "temperature": 0}).json()
        n_follow = len(tok.encode(follow))
        cached = r["timings"]["cache_n"]
        assert cached >= len(tok.encode("the quick brown fox")) and prefills[-1][1] == slot_a
        assert prefills[-1] == (n_follow - cached, slot_a, cached)
        assert r["timings"]["prompt_n"] == n_follow - cached
        nc = c.post("/completion", json={"prompt": follow, "n_predict": 5, "temperature": 0,
                                         "cache_prompt": False}).json()
        assert nc["timings"]["cache_n"] == 0 and nc["content"] == r["content"]
        # the identical prompt again: everything but its last token comes from the cache
        again = c.post("/completion", json={"prompt": follow, "n_predict": 5, "temperature": 0}).json()
        assert again["timings"]["cache_n"] == n_follow - 1 and again["content"] == r["content"]
        slots = c.get("/slots").json()
        assert len(slots) == 3 and not any(s["is_processing"] for s in slots)
        assert max(s["n_cached"] for s in slots) >= n_follow
        props = c.get("/props").json()
        assert props["total_slots"] == 3 and props["default_generation_settings"]["min_p"] == 0.05
        assert sched.metrics["prompt_tokens_cached_total"] >= 2 * cached
    finally:
        sched.close()


def test_server_penalties_and_bias_over_http(client):
    from k8s_nvidia_gpus_amd.models.llm.server import _job_from

    c, eng, tok, state = client
    sched = state["scheduler"]
    ids = tok.encode("hello")

    def run(body):
        job = sched.submit(_job_from(dict(body, temperature=0), ids, 6, eng.cfg.vocab))
        while True:
            kind, val = job.out.get(timeout=30)
            if kind == "done":
                return val.gen
            assert kind != "error", val

    plain = run({})
    banned = run({"logit_bias": [[plain[0], False]]})
    assert banned[0] != plain[0]
    pen = run({"repeat_penalty": 1e6, "repeat_last_n": -1})
    assert len(set(pen)) == len(pen) and not set(pen) & set(ids)   # nothing seen is repeated
    r = c.post("/completion", json={"prompt": "hello", "n_predict": 3, "temperature": 0,
                                    "presence_penalty": 0.5, "frequency_penalty": 0.5})
    assert r.status_code == 200
    assert c.post("/completion", json={"prompt": "hello", "logit_bias": [[10 ** 9, 1]]}).status_code == 400


def test_stream_client_gone_while_pending_is_cancelled_before_admission(tiny_model):
    """a streaming client that disconnects while its job still waits for a slot is
    noticed within a poll period; the job never gets a slot or a prefill."""
    import asyncio
    import time as _t

    from k8s_nvidia_gpus_amd.models.llm import server as S
    from k8s_nvidia_gpus_amd.models.llm.synthetic import load

    eng, tok = load(tiny_model, device="cpu", max_ctx=256, slots=1)
    real_decode = eng.decode
    eng.decode = lambda *a, **k: (_t.sleep(0.02), real_decode(*a, **k))[1]
    sched = S.Scheduler(eng, tok, parallel=1)
    try:
        busy = sched.submit(S.Job(ids=tok.encode("hello"), max_new=150))
        waiting = sched.submit(S.Job(ids=tok.encode("world"), max_new=5))

        async def gone():
            return True

        async def consume():
            out = [ev async for ev in S._astream(waiting, timeout=60, disconnected=gone)]
            return out

        t0 = _t.time()
        assert asyncio.run(consume()) == [] and _t.time() - t0 < 5
        assert waiting.cancelled and waiting.slot == -1 and waiting.gen == []
        busy.cancelled = True
    finally:
        sched.close()


def test_bad_sampler_fields_are_400_and_a_failing_sampler_ends_only_its_job(client, monkeypatch):
    """repeat_penalty=0, a non-finite temperature, top_p/min_p outside [0,1] or a bias
    banning the whole vocabulary are rejected up front; a sampler error at decode time fails only
    the job it belongs to — the request decoding next to it completes."""
    from k8s_nvidia_gpus_amd.models.llm import server as S

    c, eng, tok, state = client
    sched = state["scheduler"]
    for bad in ({"repeat_penalty": 0}, {"repeat_penalty": -1}, {"temperature": "nan"},
                {"temperature": "inf"}, {"top_p": 1.5}, {"min_p": -0.1}, {"top_k": True},
                {"logit_bias": [[i, False] for i in range(eng.cfg.vocab)]},
                {"logit_bias": [[1, "inf"]]}, {"repeat_last_n": -2}):
        r = c.post("/completion", json=dict({"prompt": "hello", "n_predict": 2}, **bad))
        assert r.status_code == 400, bad
    # a tiny temperature no longer overflows the softmax
    r = c.post("/completion", json={"prompt": "hello", "n_predict": 3, "temperature": 1e-30})
    assert r.status_code == 200
    real = S.sample_token

    def flaky(logits, p, history=(), generator=None, dist_out=None):
        if p.top_k == 7 and len(history) > len(tok.encode("boom")):   # the doomed job, in _step
            raise RuntimeError("sampler exploded")
        return real(logits, p, history, generator, dist_out=dist_out)

    monkeypatch.setattr(S, "sample_token", flaky)
    ids_a, ids_b = tok.encode("hello"), tok.encode("boom")
    a = sched.submit(S._job_from({"temperature": 0, "repeat_penalty": 1.1}, ids_a, 8, eng.cfg.vocab))
    b = sched.submit(S._job_from({"temperature": 0.7, "top_k": 7, "seed": 1}, ids_b, 8, eng.cfg.vocab))

    def result(job):
        while True:
            kind, val = job.out.get(timeout=30)
            if kind in ("done", "error"):
                return kind, val

    ka, va = result(a)
    kb, vb = result(b)
    assert ka == "done" and len(va.gen) == 8
    assert kb == "error" and "sampler exploded" in vb
    assert sched.metrics.get("requests_failed_total", 0) >= 1
    # the scheduler keeps serving
    r = c.post("/completion", json={"prompt": "again", "n_predict": 2, "temperature": 0})
    assert r.status_code == 200


def test_qwen25_embedded_template_matches_chatml_byte_for_byte():
    """the GGUF's own template renders exactly today's chatml() output."""
    from k8s_nvidia_gpus_amd.models.llm.chat_template import QWEN25_TEMPLATE, ChatFormatter
    from k8s_nvidia_gpus_amd.models.llm.tokenizer import DEFAULT_SYSTEM, chatml

    fmt = ChatFormatter(QWEN25_TEMPLATE, default_system=DEFAULT_SYSTEM)
    cases = [
        [{"role": "user", "content": "hi"}],
        [{"role": "system", "content": "Be terse."}, {"role": "user", "content": "2+2?"}],
        [{"role": "user", "content": "a"}, {"role": "assistant", "content": "b"},
         {"role": "user", "content": "c\nd"}],
        [{"role": "system", "content": "S"}, {"role": "user", "content": "u1"},
         {"role": "assistant", "content": "a1"}, {"role": "system", "content": "late system"},
         {"role": "user", "content": [{"type": "text", "text": "parts "}, {"type": "text", "text": "joined"}]}],
    ]
    for msgs in cases:
        for gen in (True, False):
            assert fmt.render(msgs, add_generation_prompt=gen) == chatml(msgs, add_generation_prompt=gen)
    # tools go through the template (the ChatML fallback has no tool format)
    out = fmt.render(cases[0], tools=[{"type": "function", "function": {"name": "f", "parameters": {}}}])
    assert "# Tools" in out and '"name": "f"' in out and out.endswith("<|im_start|>assistant\n")


LLAMA3_STYLE = ("{{- bos_token }}{% for m in messages %}<|start_header_id|>{{ m['role'] }}"
                "<|end_header_id|>\n\n{{ m['content'] | trim }}<|eot_id|>{% endfor %}"
                "{% if add_generation_prompt %}<|start_header_id|>assistant<|end_header_id|>\n\n{% endif %}")


def test_file_template_drives_chat_prompts_and_unsupported_files_are_refused(tmp_path):
    """A non-ChatML template in the file is what /v1/chat/completions uses; a Llama-architecture
    file, an unknown pre-tokeniser or a template that does not parse are refused at load."""
    from fastapi.testclient import TestClient

    from k8s_nvidia_gpus_amd.models.llm.server import Scheduler, create_app
    from k8s_nvidia_gpus_amd.models.llm.synthetic import load, write_synthetic_gguf

    p = str(tmp_path / "custom.gguf")
    write_synthetic_gguf(p, tiny(), extra_metadata={"tokenizer.chat_template": LLAMA3_STYLE})
    eng, tok = load(p, device="cpu", max_ctx=256, slots=1)
    assert tok.formatter.kind == "gguf"
    sched = Scheduler(eng, tok, parallel=1)
    try:
        c = TestClient(create_app({"scheduler": sched, "tok": tok, "model": "custom"}))
        msgs = [{"role": "user", "content": "  hello  "}]
        prompt = c.post("/apply-template", json={"messages": msgs}).json()["prompt"]
        assert prompt == ("<|endoftext|><|start_header_id|>user<|end_header_id|>\n\nhello<|eot_id|>"
                          "<|start_header_id|>assistant<|end_header_id|>\n\n")
        r = c.post("/v1/chat/completions", json={"messages": msgs, "max_tokens": 2, "temperature": 0})
        assert r.status_code == 200 and r.json()["usage"]["prompt_tokens"] == len(tok.encode(prompt))
        assert c.get("/props").json()["chat_template"] == LLAMA3_STYLE
        bad = c.post("/v1/chat/completions", json={"messages": [1, 2]})
        assert bad.status_code == 400
    finally:
        sched.close()
    for extra, needle in (({"general.architecture": "llama", "llama.block_count": 2,
                            "llama.context_length": 512, "llama.embedding_length": 256,
                            "llama.feed_forward_length": 512, "llama.attention.head_count": 2},
                           "unsupported architecture 'llama'"),
                          ({"tokenizer.ggml.pre": "deepseek-llm"}, "deepseek-llm"),
                          ({"tokenizer.chat_template": "{% for m in messages %}"}, "does not parse")):
        q = str(tmp_path / "bad.gguf")
        write_synthetic_gguf(q, tiny(), extra_metadata=extra)
        with pytest.raises(ValueError, match=needle):
            load(q, device="cpu", max_ctx=256, slots=1)


def test_gate_up_interleave_round_trip():
    """The prefill's gate|up weight layout (128-row blocks: the fused-SwiGLU GEMM's tiles hold
    matching gate and up columns): the product's columns split back into gate and up exactly."""
    from k8s_nvidia_gpus_amd.ops.llm_kernels import gate_up_interleave, gate_up_split

    torch.manual_seed(0)
    f, k = 384, 40
    wg, wu = torch.randn(f, k), torch.randn(f, k)
    w = gate_up_interleave(wg, wu)
    assert w.shape == (2 * f, k)
    assert torch.equal(w[128:256], wu[:128]) and torch.equal(w[256:384], wg[128:256])
    x = torch.randn(5, k)
    g, u = gate_up_split(x @ w.t())
    torch.testing.assert_close(g, x @ wg.t())
    torch.testing.assert_close(u, x @ wu.t())
    with pytest.raises(ValueError):
        gate_up_interleave(torch.randn(100, k), torch.randn(100, k))
