"""CPU tests of the LLM server's serving loop: chunked prompt processing
interleaved with decode steps, incremental detokenisation (host work per token independent of the
output length), stop strings across token boundaries, ``ignore_eos`` and the event-driven request
wakeups (no executor thread per waiting request)."""
import asyncio
import random
import time

import pytest
import torch

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


def _wait(job, timeout=60):
    t0 = time.time()
    while True:
        kind, val = job.out.get(timeout=max(0.1, timeout - (time.time() - t0)))
        if kind == "done":
            return val
        assert kind != "error", val


def test_stream_decoder_equals_decode(tiny_model):
    """Concatenated StreamDecoder pieces == Tokenizer.decode of the whole sequence, for random ids
    (lots of broken UTF-8), real multi-byte text cut anywhere, and control tokens in between."""
    from k8s_nvidia_gpus_amd.models.llm.tokenizer import Tokenizer, synthetic_vocab

    for tok in (_load(tiny_model)[1], Tokenizer.from_gguf(synthetic_vocab(3000))):
        rng = random.Random(0)
        words = tok.encode("naïve café 東京 🙂 ok <|im_end|> déjà vu 🎉🎉")
        for trial in range(200):
            if trial % 2:
                ids = [rng.randrange(len(tok.tokens)) for _ in range(rng.randint(1, 30))]
            else:
                ids = words[:rng.randint(1, len(words))]
            sd = tok.stream()
            pieces = [sd.push(i) for i in ids] + [sd.flush()]
            assert "".join(pieces) == tok.decode(ids), ids
            # a split multi-byte character is never streamed as U+FFFD before its last byte
            # (only the final flush of a prefix cut inside one ends as U+FFFD)
            if trial % 2 == 0:
                assert "�" not in "".join(pieces[:-1])


def test_chunked_prefill_logits_match_monolithic(tiny_model):
    eng, tok = _load(tiny_model)
    ids = tok.encode("a cozy cabin in the woods, hello world, the quick brown fox " * 3)
    full = eng.prefill(ids, slot=0)
    last = None
    for s in range(0, len(ids), 7):
        last = eng.prefill(ids[s:s + 7], slot=1, start=s)
    torch.testing.assert_close(full, last, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(eng.k_cache[:, 0, :, :len(ids)], eng.k_cache[:, 1, :, :len(ids)],
                               rtol=1e-5, atol=1e-5)


def test_prompt_chunks_interleave_with_decode_steps(tiny_model):
    """A long prompt admitted while another sequence decodes is processed ``ubatch`` tokens at a
    time, with a decode step of the running sequence between consecutive chunks; both answers
    equal their unchunked answers."""
    from k8s_nvidia_gpus_amd.models.llm import server as S

    eng, tok = _load(tiny_model)
    log = []
    real_prefill, real_decode = eng.prefill, eng.decode

    def prefill(ids, slot, start=0):
        log.append(("prefill", slot, start, len(ids)))
        return real_prefill(ids, slot, start)

    def decode(toks, pos, slots):
        log.append(("decode", tuple(slots)))
        time.sleep(0.002)
        return real_decode(toks, pos, slots)

    eng.prefill, eng.decode = prefill, decode
    long_ids = tok.encode("the quick brown fox jumps over the lazy dog. " * 6)
    assert len(long_ids) > 40
    sched = S.Scheduler(eng, tok, parallel=2, ubatch=8, batch=8)
    try:
        a = sched.submit(S.Job(ids=tok.encode("hello"), max_new=60, ignore_eos=True))
        while not a.gen:
            time.sleep(0.001)
        b = sched.submit(S.Job(ids=long_ids, max_new=4, ignore_eos=True))
        _wait(a)
        _wait(b)
    finally:
        sched.close()
    chunks = [i for i, e in enumerate(log) if e[0] == "prefill" and e[1] == b.slot]
    assert len(chunks) == -(-len(long_ids) // 8)
    assert all(log[i][3] <= 8 for i in chunks)
    assert [log[i][2] for i in chunks] == list(range(0, len(long_ids), 8))
    for i, j in zip(chunks, chunks[1:]):       # a step of the running sequence between chunks
        assert any(e[0] == "decode" and a.slot in e[1] for e in log[i + 1:j]), log[i:j + 1]
    # the same answers without chunking
    eng2, _ = _load(tiny_model)
    sched2 = S.Scheduler(eng2, tok, parallel=2, ubatch=4096)
    try:
        b2 = _wait(sched2.submit(S.Job(ids=long_ids, max_new=4, ignore_eos=True)))
        a2 = _wait(sched2.submit(S.Job(ids=tok.encode("hello"), max_new=60, ignore_eos=True)))
    finally:
        sched2.close()
    assert b.gen == b2.gen and a.gen == a2.gen and a.text == a2.text


def test_batch_size_chunks_when_nothing_decodes(tiny_model):
    from k8s_nvidia_gpus_amd.models.llm import server as S

    eng, tok = _load(tiny_model)
    sizes = []
    real = eng.prefill
    eng.prefill = lambda ids, slot, start=0: (sizes.append(len(ids)), real(ids, slot, start))[1]
    ids = tok.encode("the quick brown fox jumps over the lazy dog. " * 4)
    sched = S.Scheduler(eng, tok, parallel=1, ubatch=8, batch=32)
    try:
        _wait(sched.submit(S.Job(ids=ids, max_new=2)))
    finally:
        sched.close()
    assert sizes[0] == 32 and sum(sizes) == len(ids)


def test_prompts_of_several_slots_share_one_batch(tiny_model):
    """Prompts admitted together are processed in one prompt batch (llama-server fills a batch
    with the prompt tokens of every slot that needs them), oldest first, within the token budget;
    each answer equals the answer it gets alone."""
    from k8s_nvidia_gpus_amd.models.llm import server as S

    eng, tok = _load(tiny_model)
    calls = []
    real_many = eng.prefill_many

    def prefill_many(items):
        calls.append([(slot, start, len(ids)) for ids, slot, start in items])
        return real_many(items)

    eng.prefill_many = prefill_many
    prompts = [tok.encode(t) for t in ("a cozy cabin in the woods", "hello world, hello",
                                       "the quick brown fox jumps over the lazy dog. " * 3)]
    sched = S.Scheduler(eng, tok, parallel=3, ubatch=8, batch=24, autostart=False)
    try:
        jobs = [sched.submit(S.Job(ids=ids, max_new=6, ignore_eos=True)) for ids in prompts]
        sched.start()                                      # all three admitted in one iteration
        for j in jobs:
            _wait(j)
    finally:
        sched.close()
    first = calls[0]
    assert len(first) >= 2, calls                          # one batch, several slots
    assert sum(n for _, _, n in first) <= 24               # the batch budget
    assert [n for _, _, n in first][:2] == [len(prompts[0]), len(prompts[1])]
    for ids, j in zip(prompts, jobs):
        eng2, _ = _load(tiny_model)
        sched2 = S.Scheduler(eng2, tok, parallel=1, ubatch=4096)
        try:
            alone = _wait(sched2.submit(S.Job(ids=ids, max_new=6, ignore_eos=True)))
        finally:
            sched2.close()
        assert alone.gen == j.gen


class ScriptedEngine:
    """Engine stand-in whose greedy output is a fixed token script (positions map to script
    indices), so stop-string cases can be built from known text."""

    def __init__(self, script, vocab, prompt_len, slots=1):
        self.script, self.vocab, self.plen = list(script), vocab, prompt_len
        self.slots, self.max_ctx, self.gpu, self.device = slots, 4096, False, "cpu"

    def _at(self, pos):
        return self.script[min(pos - self.plen + 1, len(self.script) - 1)]

    def prefill(self, ids, slot, start=0):
        x = torch.zeros(self.vocab)
        x[self._at(start + len(ids) - 1)] = 1.0
        return x

    def decode_greedy(self, toks, positions, slots):
        return [self._at(p) for p in positions]


def _reference_stop(tok, gen, stops):
    """The whole-text rule applied after every token (what a server that re-decodes the output
    per token does): the first token after which some stop string occurs ends the text at the
    earliest occurrence."""
    for i in range(1, len(gen) + 1):
        text = tok.decode(gen[:i])
        hits = [text.find(s) for s in stops if s in text]
        if hits:
            return text[:min(hits)], "stop"
    return tok.decode(gen), "length"


def test_stop_strings_across_token_boundaries_and_streamed_pieces(tiny_model):
    """Stop strings found by the tail scan end the text exactly where a whole-text search after
    every token would, also when they span tokens or overlap; the streamed pieces concatenate to
    the final text."""
    from k8s_nvidia_gpus_amd.models.llm import server as S

    _, tok = _load(tiny_model)
    script = tok.encode("The answer is 42.</answer> Observation: déjà vu 🎉 more text\n\n\nend")
    prompt = tok.encode("hello")
    cases = (["</answer>"], ["answer>", "is 42"], ["42.</", "is 4"], ["vu 🎉"], ["🎉 m", "ja"],
             ["\n\n\n"], ["zzzz-not-there"], ["end"], ["Observation:", "n: d"], [""])
    for stops in cases:
        eng = ScriptedEngine(script, len(tok.tokens), len(prompt))
        sched = S.Scheduler(eng, tok, parallel=1)
        try:
            job = sched.submit(S.Job(ids=prompt, max_new=len(script), ignore_eos=True,
                                     stop=list(stops)))
            pieces = []
            while True:
                kind, val = job.out.get(timeout=30)
                if kind == "text":
                    pieces.append(val)
                elif kind == "done":
                    break
        finally:
            sched.close()
        want, reason = _reference_stop(tok, script, stops)
        assert (val.text, val.finish) == (want, reason), stops
        assert "".join(pieces) == want


def test_ignore_eos_runs_to_n_predict(tiny_model):
    from k8s_nvidia_gpus_amd.models.llm import server as S

    eng, tok = _load(tiny_model)
    eos = sorted(tok.stop_ids())[0]
    sched = S.Scheduler(eng, tok, parallel=1)
    try:
        # a logit bias that forces the stop token: without ignore_eos the job ends at once
        from k8s_nvidia_gpus_amd.models.llm.sampling import SamplingParams

        p = SamplingParams.from_request({"temperature": 0, "logit_bias": [[eos, 100.0]]},
                                        eng.cfg.vocab)
        a = _wait(sched.submit(S.Job(ids=tok.encode("hi"), max_new=5, params=p)))
        b = _wait(sched.submit(S.Job(ids=tok.encode("hi"), max_new=5, params=p, ignore_eos=True)))
    finally:
        sched.close()
    assert a.gen == [eos] and a.finish == "stop"
    assert len(b.gen) == 5 and b.finish == "length" and b.text == ""


def test_host_time_per_token_is_flat_in_output_length(tiny_model, monkeypatch):
    """``_emit`` used to re-decode the whole output per token.  Now the full decoder
    is never called while streaming, and per-token host time at 2048 generated tokens is within
    a small factor of the time at 16."""
    from k8s_nvidia_gpus_amd.models.llm import server as S

    eng, tok = _load(tiny_model)
    sched = S.Scheduler(eng, tok, parallel=1)
    sched.close()                        # only _emit is exercised, on this thread
    monkeypatch.setattr(type(tok), "decode", lambda *a, **k: pytest.fail("full re-decode"))
    rng = random.Random(1)
    normal = [i for i in range(len(tok.tokens)) if i not in tok.special_ids]
    job = S.Job(ids=[1, 2, 3], max_new=10 ** 6, stop=["</answer>", "\n\n\n\n", "Observation:"])
    job.detok = tok.stream()

    def per_token(n):
        toks = [rng.choice(normal) for _ in range(n)]
        t0 = time.perf_counter()
        for t in toks:
            assert not sched._emit(job, t) or job.finish == "stop"
            if job.finish:
                job.finish = ""
        return (time.perf_counter() - t0) / n

    per_token(16)
    early = min(per_token(16) for _ in range(5))
    while len(job.gen) < 2048:
        per_token(256)
    late = min(per_token(16) for _ in range(5))
    assert len(job.gen) >= 2048
    assert late < 3 * early + 20e-6, (early, late)
    while not job.out.empty():
        job.out.get_nowait()


def test_waiting_requests_hold_no_executor_thread(tiny_model):
    """16 concurrent streams in one event loop whose default executor refuses work —
    every stream completes, woken by the scheduler rather than by executor polls."""
    from concurrent.futures import ThreadPoolExecutor

    from k8s_nvidia_gpus_amd.models.llm import server as S

    eng, tok = _load(tiny_model, slots=4)
    sched = S.Scheduler(eng, tok, parallel=4, ubatch=4)

    class NoThreads(ThreadPoolExecutor):
        def submit(self, *a, **k):
            raise AssertionError("a waiting request used an executor thread")

    async def main():
        asyncio.get_running_loop().set_default_executor(NoThreads(1))
        jobs = [sched.submit(S.Job(ids=tok.encode(f"hello {i}"), max_new=6, ignore_eos=True))
                for i in range(16)]

        async def consume(j):
            return [k async for k, _ in S._astream(j, timeout=60)]
        return await asyncio.gather(*(consume(j) for j in jobs))

    try:
        outs = asyncio.run(main())
    finally:
        sched.close()
    assert all(o[-1] == "done" for o in outs)


def test_prefill_many_equals_one_by_one_and_validates(tiny_model):
    """``Engine.prefill_many`` off the GPU prompt path runs the chunks one after the other: the
    same logits and KV as separate prefills; an empty chunk or one past the context is rejected."""
    eng, tok = _load(tiny_model, slots=4)
    a, b = tok.encode("a cozy cabin in the woods"), tok.encode("hello world")
    got = eng.prefill_many([(a, 0, 0), (b, 1, 0)])
    eng2, _ = _load(tiny_model, slots=4)
    want = [eng2.prefill(a, 0), eng2.prefill(b, 1)]
    for g, w in zip(got, want):
        torch.testing.assert_close(g, w)
    torch.testing.assert_close(eng.k_cache[:, :2], eng2.k_cache[:, :2])
    with pytest.raises(ValueError):
        eng.prefill_many([(a, 2, 0), ([], 3, 0)])
    with pytest.raises(ValueError):
        eng.prefill_many([(a, 2, 0), (b, 3, eng.max_ctx - 1)])


def test_short_prompts_fitting_the_batch_are_taken_whole_while_decoding(tiny_model):
    """While a sequence decodes, prompts whose rest fits the batch budget are prefilled whole in
    one iteration (a burst of requests starts decoding together); a prompt that does not fit is
    still cut into ubatch chunks."""
    from k8s_nvidia_gpus_amd.models.llm import server as S

    eng, tok = _load(tiny_model)
    calls = []
    real_many, real_prefill = eng.prefill_many, eng.prefill

    def prefill_many(items):
        calls.append([len(ids) for ids, _, _ in items])
        return real_many(items)

    def prefill(ids, slot, start=0):
        calls.append([len(ids)])
        return real_prefill(ids, slot, start)

    real_decode = eng.decode

    def decode(toks, pos, slots):
        time.sleep(0.002)                  # keep the first sequence decoding throughout
        return real_decode(toks, pos, slots)

    eng.prefill_many, eng.prefill, eng.decode = prefill_many, prefill, decode
    sched = S.Scheduler(eng, tok, parallel=4, ubatch=8, batch=64)
    try:
        a = sched.submit(S.Job(ids=tok.encode("hello"), max_new=150, ignore_eos=True))
        while not a.gen:
            time.sleep(0.001)
        n0 = len(calls)
        short = [tok.encode(t) for t in ("a cozy cabin in the woods by a river",
                                         "the quick brown fox jumps over it")]
        assert all(8 < len(ids) <= 32 for ids in short)
        jobs = [sched.submit(S.Job(ids=ids, max_new=3, ignore_eos=True)) for ids in short]
        longer = tok.encode("the lazy dog sleeps in the sun all day long. " * 6)
        assert len(longer) > 64
        c = sched.submit(S.Job(ids=longer, max_new=3, ignore_eos=True))
        for j in jobs + [c]:
            _wait(j)
        assert not a.finish                      # it decoded all along
        _wait(a)
    finally:
        sched.close()
    later = [n for batch in calls[n0:] for n in batch]
    assert len(short[0]) in later and len(short[1]) in later       # each taken whole
    # the long one in ubatch chunks, down to its last one
    assert 8 * sum(1 for n in later if n == 8) >= len(longer) - 8


class ChainedStepEngine:
    """CPU engine wrapper whose greedy steps are chainable, as the GPU engine's are: a chained
    step reads its tokens from the in-flight step (``decode_greedy_async(None, ..., chain=)``)."""

    def __init__(self, eng):
        self._eng = eng
        self.calls = []

    def __getattr__(self, name):
        return getattr(self._eng, name)

    def decode_greedy_async(self, tokens, positions, slots, chain=None):
        from types import SimpleNamespace

        from k8s_nvidia_gpus_amd.models.llm.engine import GreedyStep

        self.calls.append("chained" if tokens is None else "host")
        if tokens is None:
            assert chain is not None and chain.chainable and chain.buffers.T == len(positions)
            tokens = chain.result()
        step = GreedyStep(value=self._eng.decode_greedy(tokens, positions, slots))
        step.chainable, step.buffers = True, SimpleNamespace(T=len(positions))
        return step


def test_pipelined_greedy_steps_give_the_unpipelined_answers(tiny_model):
    """Greedy steps of an unchanged batch are enqueued back to back, the next one fed on the
    in-flight step's tokens; sequences finishing mid-chain (different max_new, a stop string)
    get no extra token, and every answer equals the one-step-at-a-time scheduler's."""
    from k8s_nvidia_gpus_amd.models.llm import server as S

    eng, tok = _load(tiny_model)
    prompts = [tok.encode(t) for t in ("a cozy cabin", "hello world", "the lazy dog", "one two")]
    lens = [5, 17, 9, 30]

    def run(pipeline, engine):
        sched = S.Scheduler(engine, tok, parallel=4, ubatch=64, autostart=False, pipeline=pipeline)
        try:
            jobs = [sched.submit(S.Job(ids=ids, max_new=n, ignore_eos=True))
                    for ids, n in zip(prompts, lens)]
            sched.start()
            return [_wait(j) for j in jobs], sched
        finally:
            sched.close()

    chained = ChainedStepEngine(eng)
    got, sched = run(True, chained)
    eng2, _ = _load(tiny_model)
    want, _ = run(False, eng2)
    for g, w, n in zip(got, want, lens):
        assert g.gen == w.gen and len(g.gen) == n and g.text == w.text
    assert chained.calls.count("chained") > 10                 # the steps did chain
    assert sched.metrics["tokens_predicted_total"] == sum(lens)
