"""llama-server-compatible HTTP API over the in-tree Qwen2 engine, with continuous batching.

The reference's LLM pod runs ``llama-server -m <gguf> --host 0.0.0.0 --port 8080 --ctx-size 4096
--n-gpu-layers 35 --threads 6`` behind Service ``coder-llm`` and a Gateway (reference
cluster-config/apps/llm/deployment.yaml:76-84, service.yaml, httproute.yaml).  This server accepts
the same command line (``-m``, ``--ctx-size``, ``--n-gpu-layers`` / ``--threads`` accepted; every
layer is on the GPU) and serves the endpoints clients of that pod use:

* ``GET /health`` (503 while the model loads, like llama-server), ``GET /v1/models``;
* ``POST /completion`` (llama.cpp native: ``prompt``, ``n_predict``, ``seed``, ``stop``,
  ``stream``, ``cache_prompt`` and the sampler fields of ``sampling.py`` — temperature, top_k,
  top_p, min_p, repeat_penalty / repeat_last_n, presence / frequency penalty, logit_bias) with
  llama.cpp's ``timings`` block; ``n_probs`` (+ ``post_sampling_probs``) adds llama-server's
  ``completion_probabilities``; ``grammar`` (GBNF), ``json_schema`` and ``response_format``
  constrain the output (grammar.py) — OpenAI's ``logprobs`` / ``top_logprobs`` likewise.  A field
  the server cannot honour (``n`` > 1, a schema keyword outside grammar.py's subset) is answered
  with HTTP 400 naming it, never silently ignored;
* ``POST /v1/completions`` and ``POST /v1/chat/completions`` (OpenAI; the prompt is rendered with
  the model file's own ``tokenizer.chat_template`` — chat_template.py — ChatML when it has none;
  ``tools`` are passed to the template; ``stream`` as server-sent events);
* ``POST /apply-template``, ``POST /tokenize``, ``POST /detokenize``, ``GET /props``, ``GET /slots``,
  ``GET /metrics`` (Prometheus text).

Request sampler fields are range-checked (400 on a non-finite temperature, ``repeat_penalty <= 0``,
``top_p`` / ``min_p`` outside [0, 1], a bias that bans the whole vocabulary …); a sampler failure
at decode time ends only the request it belongs to.  Prompt tokenisation and template rendering
run in the thread pool, never on the event loop.

One scheduler thread owns the GPU: new requests take free KV-cache slots and their prompts are
processed between the decode steps of the sequences already generating — prompts that fit the
``--batch-size`` budget whole, a longer one in chunks of ``--ubatch-size`` tokens, one chunk per
loop iteration — up to 8 sequences share each pass over the weights
(``--parallel``).  Request handlers await per-request events that the scheduler sets, so the GPU is
never driven from two threads (the reference's SD15 app had that hazard).  A request
whose client goes away (stream closed, or the connection dropped while a blocking request waits)
is cancelled and frees its KV slot at the next decode step; a request whose prefill or first
sample fails gets that error, and no handler waits longer than ``--timeout`` seconds.

Prompt caching (llama-server's ``cache_prompt``, on by default): every slot remembers which tokens
its KV cache holds; a new request goes to the free slot sharing the longest prefix with its
prompt, and only the rest of the prompt is prefilled (multi-turn chats re-send the whole history).
As with llama-server, a reused prefix was computed in another prefill (a GEMM of another M), so
the logits can differ in the last bits from an uncached prefill of the same prompt.  Prompts
admitted in the same iteration are prefilled together (one GEMM over all their rows), so the same
holds with concurrent traffic: a seeded or greedy request can differ in the last bits, and rarely
in a token, depending on which prompts arrived with it — ``--no-prompt-batch`` prefills every
prompt alone for runs that must reproduce exactly.  Decode itself is batch-invariant.
"""
from __future__ import annotations

import argparse
import asyncio
import collections
import gc
import json
import math
import os
import queue
import threading
import time
import uuid
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

import torch

from .engine import Engine
from .sampling import SamplingParams, sample_token
from .tokenizer import Tokenizer

try:   # module level: FastAPI resolves the handlers' (postponed) annotations in this namespace
    from fastapi import Request
except ImportError:  # pragma: no cover - the engine/scheduler work without the HTTP layer
    Request = None


@dataclass
class Job:
    ids: List[int]
    max_new: int
    params: SamplingParams = field(default_factory=SamplingParams)
    seed: Optional[int] = None
    cache_prompt: bool = True
    stop: List[str] = field(default_factory=list)
    ignore_eos: bool = False
    out: "queue.Queue" = field(default_factory=queue.Queue)
    # scheduler state
    slot: int = -1
    pos: int = 0               # tokens whose KV the slot holds: prompt progress, then + generated
    decoding: bool = False     # the prompt is done; the job takes one token per decode step
    last: int = 0
    gen: List[int] = field(default_factory=list)
    parts: List[str] = field(default_factory=list)   # emitted text pieces
    tail: str = ""             # decoded but held back: it may be the start of a stop string
    detok: Any = None          # tokenizer.StreamDecoder of this job
    generator: Optional[torch.Generator] = None
    t_submit: float = 0.0
    t_first: float = 0.0
    t_prefill: float = 0.0
    finish: str = ""
    cancelled: bool = False
    n_cached: int = 0          # prompt tokens whose KV was reused from the slot
    waker: Any = None          # (event loop, asyncio.Event) of the coroutine waiting on ``out``
    grammar: Any = None        # grammar.GrammarState: constrained decoding (grammar / JSON)
    n_probs: int = 0           # top-n probabilities per generated token (n_probs / logprobs)
    want_probs: bool = False   # record each generated token's probability entry
    post_probs: bool = False   # entries from the sampler's final distribution, not the logits
    probs: List[dict] = field(default_factory=list)

    @property
    def fast_greedy(self) -> bool:
        """argmax of the raw logits is all this job needs (the in-graph greedy step applies)."""
        return self.params.plain_greedy and self.grammar is None and not self.want_probs

    @property
    def text(self) -> str:
        return "".join(self.parts)


def common_prefix(a: List[int], b: List[int]) -> int:
    n = min(len(a), len(b))
    i = 0
    while i < n and a[i] == b[i]:
        i += 1
    return i


def _set_events(events) -> None:
    for e in events:
        e.set()


class Scheduler:
    """Continuous batching over the engine's KV-cache slots, with chunked prompt processing.

    One loop iteration: admit pending requests into free slots → one prompt batch → one decode
    step of every sequence whose prompt is done → wake the consumers.  The prompt batch takes the
    admitted prompts oldest first: every prompt whose rest fits the ``batch`` budget
    (llama-server's ``n_batch``) whole, so a burst of requests starts decoding together, and of a
    prompt that does not fit one chunk — at most ``ubatch`` tokens while other sequences decode.
    A long prompt therefore stalls the running streams for one chunk at a time, not for its whole
    prefill (llama-server's update loop fills one n_batch with the decoding slots' tokens and the
    prompt tokens; reference cluster-config/apps/llm/deployment.yaml:61,76-84 runs llama-server).

    Host work per generated token is independent of the length of the output: each token is
    detokenised alone (``StreamDecoder``: incomplete UTF-8 carried over) and the stop strings are
    searched only in the held-back tail plus the new text."""

    def __init__(self, engine: Engine, tok: Tokenizer, parallel: int = 8, ubatch: int = 512,
                 batch: Optional[int] = None, autostart: bool = True, prompt_batch: bool = True,
                 pipeline: bool = True):
        self.engine = engine
        self.tok = tok
        # prompt chunks of several slots in one pass (engine.prefill_many): its GEMMs run at an M
        # that depends on which prompts arrived together, so a prompt's logits can differ in the
        # last bits with the traffic; False prefills every prompt alone (--no-prompt-batch), for
        # runs that must reproduce bit for bit
        self.prompt_batch = prompt_batch
        # greedy steps of an unchanged batch enqueued back to back (_step_pipelined); False: every
        # step waits for its tokens before the next one is enqueued
        self.pipeline = pipeline
        self._inflight = None                            # (jobs, GreedyStep, t0) of the step in flight
        self.parallel = max(1, min(parallel, engine.slots))
        self.ubatch = max(1, int(ubatch))
        self.batch = max(self.ubatch, int(batch or self.ubatch))
        self.pending: "queue.Queue[Job]" = queue.Queue()
        self.active: Dict[int, Job] = {}                 # slot -> job (prompt or decode phase)
        self.prefilling: List[Job] = []                  # admitted, prompt not done (FIFO)
        self.slot_tokens: Dict[int, List[int]] = {}      # tokens whose KV each free slot holds
        self.stop_ids = set(tok.stop_ids())
        self.metrics = {"requests_total": 0, "prompt_tokens_total": 0, "tokens_predicted_total": 0,
                        "decode_steps_total": 0, "decode_seconds_total": 0.0,
                        "prefill_seconds_total": 0.0, "prefill_chunks_total": 0,
                        "prefill_batches_total": 0,
                        "requests_processing": 0, "prompt_tokens_cached_total": 0}
        self._touched: List[Job] = []
        # per-iteration timings (GET /debug/iterations): start, admit / prefill / step / wake
        # seconds, prompt tokens processed, sequences decoded; and the interpreter's GC pauses
        self.trace: "collections.deque" = collections.deque(maxlen=8192)
        self.gc_pauses: "collections.deque" = collections.deque(maxlen=1024)
        self._gc_t0 = 0.0
        gc.callbacks.append(self._gc_cb)
        self._run = True
        self._lock = threading.Lock()
        self.thread = threading.Thread(target=self._loop, name="llm-scheduler", daemon=True)
        if autostart:
            self.thread.start()

    def start(self) -> None:
        """Start the scheduler thread (``autostart=False``: after queueing requests, e.g. so that
        several are admitted in one iteration)."""
        if not self.thread.is_alive():
            self.thread.start()

    def submit(self, job: Job) -> Job:
        if len(job.ids) == 0:
            raise ValueError("empty prompt")
        if len(job.ids) + 1 >= self.engine.max_ctx:
            raise ValueError(f"prompt of {len(job.ids)} tokens exceeds the context "
                             f"({self.engine.max_ctx})")
        job.max_new = max(1, min(job.max_new, self.engine.max_ctx - len(job.ids) - 1))
        job.t_submit = time.perf_counter()
        with self._lock:
            self.metrics["requests_total"] += 1
        self.pending.put(job)
        return job

    def _gc_cb(self, phase, info) -> None:
        if phase == "start":
            self._gc_t0 = time.perf_counter()
        else:
            self.gc_pauses.append((self._gc_t0, time.perf_counter() - self._gc_t0,
                                   info.get("generation", -1)))

    def close(self) -> None:
        try:
            gc.callbacks.remove(self._gc_cb)
        except ValueError:
            pass
        self._run = False
        self.pending.put(None)  # type: ignore[arg-type]
        if self.thread.is_alive():
            self.thread.join(timeout=10)

    # ---------------------------------------------------------------- scheduler thread
    def _put(self, job: Job, item) -> None:
        job.out.put(item)
        self._touched.append(job)

    def _wake(self) -> None:
        """One ``call_soon_threadsafe`` per event loop for everything this iteration produced."""
        if not self._touched:
            return
        by_loop: Dict[Any, list] = {}
        for j in self._touched:
            w = j.waker
            if w is not None:
                by_loop.setdefault(w[0], []).append(w[1])
        self._touched = []
        for loop, events in by_loop.items():
            try:
                loop.call_soon_threadsafe(_set_events, events)
            except RuntimeError:      # that loop has closed: nobody is waiting any more
                pass

    def _free_slot(self, ids: Optional[List[int]] = None) -> int:
        """A free slot: the one whose cached tokens share the longest prefix with ``ids``, else
        the one with the least cached context (keeps other conversations' caches warm)."""
        free = [s for s in range(self.parallel) if s not in self.active]
        if not free:
            return -1
        def key(s):
            held = self.slot_tokens.get(s, [])
            return (common_prefix(held, ids) if ids else 0, -len(held), -s)
        return max(free, key=key)

    def _release(self, job: Job) -> None:
        """Forget ``job``'s slot assignment; its KV (the first ``pos`` tokens) stays reusable."""
        if job.slot < 0:
            return
        self.slot_tokens[job.slot] = (job.ids + job.gen)[:job.pos]
        if self.active.get(job.slot) is job:
            del self.active[job.slot]

    def _fail(self, job: Job, e: Exception) -> None:
        with self._lock:
            self.metrics["requests_failed_total"] = self.metrics.get("requests_failed_total", 0) + 1
        self._put(job, ("error", repr(e)))
        self._release(job)

    @staticmethod
    def _recent(job: Job) -> List[int]:
        """The history the sampler's repetition penalties look at (``repeat_last_n`` tokens of
        prompt + output; all of it for -1) — not a copy of the whole sequence per token."""
        n = job.params.repeat_last_n
        if n < 0:
            return job.ids + job.gen
        if n == 0:
            return []
        g = job.gen[-n:]
        if len(g) == n:
            return g
        return job.ids[max(0, len(job.ids) - (n - len(g))):] + g

    def _sample(self, job: Job, logits: torch.Tensor) -> int:
        """The job's next token from ``logits`` [vocab]: its sampler chain, under its grammar as
        llama.cpp's common sampler does (keep the draw when the grammar accepts it, else mask
        every rejected token and draw again), and its probability entry when it asked for one."""
        dist: Optional[dict] = {} if job.post_probs else None
        hist = self._recent(job)
        tok = sample_token(logits, job.params, hist, job.generator, dist_out=dist)
        g = job.grammar
        if g is not None and not g.accepts(tok):
            mask = g.mask(logits.numel(), logits.device)
            if not bool(mask.any()):
                from .grammar import GrammarError

                raise GrammarError("no token of the vocabulary can continue the grammar here")
            tok = sample_token(logits.masked_fill(~mask, -float("inf")), job.params, hist,
                               job.generator, dist_out=dist)
        if g is not None:
            g.advance(tok)
        if job.want_probs:
            entry = self._probs_entry(job, logits, tok, dist)
            job.probs.append(entry)
            self._put(job, ("probs", entry))
        return tok

    def _piece(self, tid: int) -> dict:
        bs = self.tok.token_bytes()[tid] if 0 <= tid < len(self.tok.token_bytes()) else b""
        return {"id": tid, "token": bs.decode("utf-8", "replace") if bs else
                self.tok.decode([tid], skip_special=False), "bytes": list(bs)}

    def _probs_entry(self, job: Job, logits: torch.Tensor, tok: int, dist) -> dict:
        """llama-server's per-token entry: the token, its log-probability under the model's
        softmax (or, post_probs, its probability in the sampler's final distribution) and the
        n most likely alternatives."""
        if job.post_probs:
            p = dist["probs"].float()
            k = min(job.n_probs, int((p > 0).sum().item())) if job.n_probs else 0
            top = torch.topk(p, k) if k else None
            e = dict(self._piece(tok), prob=float(p[tok].item()))
            e["top"] = ([dict(self._piece(int(i)), prob=float(v)) for v, i in
                         zip(top.values.tolist(), top.indices.tolist())] if top is not None else [])
            return e
        lp = torch.log_softmax(logits.float(), -1)
        top = torch.topk(lp, min(job.n_probs, lp.numel())) if job.n_probs else None
        e = dict(self._piece(tok), logprob=float(lp[tok].item()))
        e["top"] = ([dict(self._piece(int(i)), logprob=float(v)) for v, i in
                     zip(top.values.tolist(), top.indices.tolist())] if top is not None else [])
        return e

    def _emit(self, job: Job, tok: int) -> bool:
        """Record a sampled token; returns True when the job is finished."""
        job.gen.append(tok)
        job.last = tok
        if tok in self.stop_ids and not job.ignore_eos:
            job.finish = "stop"
            self._flush(job, job.detok.flush(), final=True)
            return True
        new = job.detok.push(tok)
        if job.grammar is not None and job.grammar.finished:
            # the grammar admits nothing but the end: the answer is complete
            job.finish = "stop"
            self._flush(job, new + job.detok.flush(), final=True)
            return True
        if len(job.gen) >= job.max_new:
            job.finish = "length"
            self._flush(job, new + job.detok.flush(), final=True)
            return True
        return self._flush(job, new, final=False)

    def _flush(self, job: Job, new: str, final: bool) -> bool:
        """Emit ``job.tail + new`` up to a stop string (then the job ends, reason "stop"), holding
        back a suffix that may still grow into one.  Returns True when a stop string ended it."""
        s = job.tail + new
        cut = -1
        for st in job.stop:
            i = s.find(st)
            if i >= 0 and (cut < 0 or i < cut):
                cut = i
        hold = 0
        if cut >= 0:
            s, final = s[:cut], True
            job.finish = "stop"
        elif not final:
            for st in job.stop:                  # a stop string may be starting: hold its prefix
                for k in range(min(len(st) - 1, len(s)), hold, -1):
                    if s.endswith(st[:k]):
                        hold = k
                        break
        piece, job.tail = s[:len(s) - hold], s[len(s) - hold:]
        if piece:
            job.parts.append(piece)
            self._put(job, ("text", piece))
        if final:
            self._put(job, ("done", job))
        return cut >= 0

    def _admit(self) -> None:
        while len(self.active) < self.parallel:
            try:
                job = self.pending.get_nowait() if self.active else self.pending.get(timeout=0.5)
            except queue.Empty:
                return
            if job is None:
                return
            if job.cancelled:
                continue
            slot = self._free_slot(job.ids if job.cache_prompt else None)
            try:
                if job.params.temperature > 0:
                    dev = self.engine.device if self.engine.gpu else "cpu"
                    job.generator = torch.Generator(device=dev)
                    job.generator.manual_seed(job.seed if job.seed is not None
                                              else int.from_bytes(os.urandom(4), "little"))
                job.detok = self.tok.stream()
            except Exception as e:  # noqa: BLE001 - this job fails; the others keep going
                self._fail(job, e)
                continue
            # reuse the slot's KV for the shared prefix; at least one token is prefilled (its
            # logits are the first sample)
            n_past = 0
            if job.cache_prompt:
                n_past = min(common_prefix(self.slot_tokens.get(slot, []), job.ids),
                             len(job.ids) - 1)
            self.slot_tokens[slot] = []                 # the KV is being rewritten
            job.slot, job.pos, job.n_cached = slot, n_past, n_past
            self.active[slot] = job
            self.prefilling.append(job)

    def _prefill_chunk(self) -> int:
        """One prompt batch: chunks of the admitted prompts, oldest first, up to the batch's
        token budget (``ubatch`` while other sequences decode, ``batch`` otherwise) — like
        llama-server, which fills one batch with the prompt tokens of every slot that needs them.
        A prompt's last chunk samples its first token.  Returns the number of prompt tokens."""
        for j in [j for j in self.prefilling if j.cancelled]:
            self.prefilling.remove(j)
            self._release(j)
        if not self.prefilling:
            return 0
        # a decode step still in flight finishes first: the prompt batch's wall time (one sync)
        # then covers the prompt work only
        self._flush_inflight()
        # Prompts that fit the batch (``batch`` tokens, llama-server's n_batch) whole are taken
        # whole: a burst of new requests all start decoding within an iteration or two.  A prompt
        # that does not fit is cut into chunks — of at most ``ubatch`` tokens while other
        # sequences decode, down to its last one (its tail is not taken whole either), so a long
        # prompt stalls the running streams one ubatch at a time.
        decoding = any(j.decoding for j in self.active.values())
        budget = self.batch
        work = []
        for job in self.prefilling:
            rem = len(job.ids) - job.pos
            if rem <= 0:
                break
            if rem <= budget and (not decoding or job.pos == job.n_cached):
                work.append((job, rem))
                budget -= rem
                if budget == 0:
                    break
                continue
            if not decoding:
                work.append((job, min(rem, budget)))
            elif not work:
                work.append((job, min(rem, budget, self.ubatch)))
            break
        t0 = time.perf_counter()
        many = getattr(self.engine, "prefill_many", None) if self.prompt_batch else None
        results = {}
        if many is not None and len(work) > 1:
            try:
                out = many([(job.ids[job.pos:job.pos + n], job.slot, job.pos) for job, n in work])
                results = {id(job): lg for (job, _), lg in zip(work, out)}
            except Exception:  # noqa: BLE001 - retried one by one below, so only the bad one fails
                results = {}
        total = 0
        charged = []
        for job, n in work:
            try:
                logits = results.get(id(job))
                if logits is None:
                    logits = self.engine.prefill(job.ids[job.pos:job.pos + n], job.slot,
                                                 start=job.pos)
                done = job.pos + n == len(job.ids)
                tok = self._sample(job, logits) if done else None
            except Exception as e:  # noqa: BLE001 - this job fails; the others keep decoding
                self.prefilling.remove(job)
                self._fail(job, e)
                continue
            job.pos += n
            total += n
            charged.append((job, n))
            with self._lock:
                self.metrics["prompt_tokens_total"] += n
                self.metrics["prefill_chunks_total"] += 1
            if not done:
                continue
            self.prefilling.remove(job)
            job.t_first = time.perf_counter()
            job.decoding = True
            with self._lock:
                self.metrics["prompt_tokens_cached_total"] += job.n_cached
                self.metrics["tokens_predicted_total"] += 1
            if self._emit(job, int(tok)):
                self._release(job)
        if work:
            # The prompt work is asynchronous on the GPU: without a sync here it would be charged
            # to the next decode step's host sync (a 30k-token prompt read 220 ms of prompt time
            # for ~0.8 s of chunks).  The batch's wall time counts once; each job is
            # charged its token share of it.
            if getattr(self.engine, "gpu", False):
                torch.cuda.synchronize()
            wall = time.perf_counter() - t0
            for job, n in charged:
                job.t_prefill += wall * n / max(total, 1)
            with self._lock:
                self.metrics["prefill_seconds_total"] += wall
                self.metrics["prefill_batches_total"] += 1
        return total

    def _consume(self, jobs: List[Job], toks: List[int]) -> int:
        """Tokens of a finished step: advance, emit, release the finished.  A job that left
        the batch while the step was in flight (finished or cancelled) gets nothing."""
        n = 0
        for j, t in zip(jobs, toks):
            if self.active.get(j.slot) is not j or not j.decoding:
                continue
            j.pos += 1          # the step wrote this job's KV
            n += 1
            if self._emit(j, int(t)):
                self._release(j)
        with self._lock:
            self.metrics["tokens_predicted_total"] += n
        return n

    def _flush_inflight(self) -> int:
        """Wait for the step in flight (if any) and hand out its tokens."""
        infl, self._inflight = self._inflight, None
        if infl is None:
            return 0
        jobs, step, t0 = infl
        toks = step.result()
        with self._lock:
            self.metrics["decode_seconds_total"] += time.perf_counter() - t0
        return self._consume(jobs, toks)

    def _step_pipelined(self, jobs: List[Job]) -> int:
        """Greedy steps of an unchanged batch run back to back on the GPU: the next step is
        enqueued (its tokens read on the GPU from the in-flight step's ids) before the in-flight
        step's tokens are detokenised and sent, so the host work of a step hides under the next
        one.  When the batch changes, the in-flight step is flushed first."""
        infl = self._inflight
        if infl is not None and [id(j) for j in infl[0]] == [id(j) for j in jobs] and \
                infl[1].chainable:
            t0 = time.perf_counter()
            nxt = self.engine.decode_greedy_async(None, [j.pos + 1 for j in jobs],
                                                  [j.slot for j in jobs], chain=infl[1])
            with self._lock:
                self.metrics["decode_steps_total"] += 1
            n = self._flush_inflight()
            self._inflight = (jobs, nxt, t0)
            return n
        n = self._flush_inflight()
        jobs = [j for j in self.active.values() if j.decoding and not j.cancelled]
        if not jobs or not all(j.fast_greedy for j in jobs):
            return n
        t0 = time.perf_counter()
        step = self.engine.decode_greedy_async([j.last for j in jobs], [j.pos for j in jobs],
                                               [j.slot for j in jobs])
        with self._lock:
            self.metrics["decode_steps_total"] += 1
        self._inflight = (jobs, step, t0)
        return n

    def _step(self) -> int:
        """One decode step of every sequence past its prompt; returns how many tokens were
        handed out."""
        for j in [j for j in self.active.values() if j.decoding and j.cancelled]:
            self._release(j)
        jobs = [j for j in self.active.values() if j.decoding]
        if not jobs:
            return self._flush_inflight()
        if self.pipeline and all(j.fast_greedy for j in jobs) and \
                hasattr(self.engine, "decode_greedy_async"):
            return self._step_pipelined(jobs)
        n_flushed = self._flush_inflight()
        jobs = [j for j in self.active.values() if j.decoding]
        if not jobs:
            return n_flushed
        t0 = time.perf_counter()
        args = ([j.last for j in jobs], [j.pos for j in jobs], [j.slot for j in jobs])
        if all(j.fast_greedy for j in jobs) and hasattr(self.engine, "decode_greedy"):
            toks = self.engine.decode_greedy(*args)       # argmax inside the step's graph
        else:
            logits = self.engine.decode(*args)
            toks = []
            for i, j in enumerate(jobs):
                try:   # a request's own sampler failure ends that request only
                    toks.append(self._sample(j, logits[i]))
                except Exception as e:  # noqa: BLE001
                    toks.append(e)
        dt = time.perf_counter() - t0
        with self._lock:
            self.metrics["decode_steps_total"] += 1
            self.metrics["decode_seconds_total"] += dt
            self.metrics["tokens_predicted_total"] += sum(1 for t in toks if not isinstance(t, Exception))
        for j, t in zip(jobs, toks):
            j.pos += 1          # the step wrote this job's KV either way
            if isinstance(t, Exception):
                self._fail(j, t)
            elif self._emit(j, int(t)):
                self._release(j)
        return n_flushed + len(jobs)

    def _loop(self) -> None:
        clock = time.perf_counter
        while self._run:
            try:
                t0 = clock()
                self._admit()
                self.metrics["requests_processing"] = len(self.active)
                t1 = clock()
                n_prompt = self._prefill_chunk()
                t2 = clock()
                self._wake()                 # a finished prompt's first token goes out now
                t3 = clock()
                n_dec = self._step()
                t4 = clock()
                self._wake()
                if n_prompt or n_dec:
                    self.trace.append((t0, t1 - t0, t2 - t1, t4 - t3, clock() - t4 + t3 - t2,
                                       n_prompt, n_dec))
            except Exception as e:  # surface to every waiting request, keep serving
                for j in list(self.active.values()):
                    self._put(j, ("error", repr(e)))
                self.active.clear()
                self.prefilling.clear()
                self.slot_tokens.clear()
                self._wake()


# -------------------------------------------------------------------- HTTP layer
def _int_field(body: Dict[str, Any], key: str, lo: int, hi: int) -> Optional[int]:
    v = body.get(key)
    if v is None:
        return None
    if isinstance(v, bool) or not isinstance(v, int) or not lo <= v <= hi:
        raise ValueError(f"{key} must be an integer in [{lo}, {hi}], got {v!r}")
    return v


def _probs_request(body: Dict[str, Any], api: str, vocab: Optional[int]) -> tuple:
    """(record entries, top-n, post-sampling) from llama-server's ``n_probs`` /
    ``post_sampling_probs`` or OpenAI's ``logprobs`` (+ ``top_logprobs`` for chat)."""
    vmax = int(vocab or 1 << 20)
    post = body.get("post_sampling_probs")
    if post is not None and not isinstance(post, bool):
        raise ValueError("post_sampling_probs must be a boolean")
    if api == "chat":
        lp = body.get("logprobs")
        if lp is not None and not isinstance(lp, bool):
            raise ValueError("logprobs must be a boolean for chat completions")
        top = _int_field(body, "top_logprobs", 0, 20)
        if top is not None and not lp:
            raise ValueError("top_logprobs needs logprobs: true")
        n = _int_field(body, "n_probs", 0, vmax) or 0
        return bool(lp) or n > 0, (top if top is not None else n), bool(post)
    if api == "completions":
        lp = body.get("logprobs")
        if lp is not None and (isinstance(lp, bool) or not isinstance(lp, int) or lp < 0
                               or lp > min(vmax, 100)):
            raise ValueError("logprobs must be an integer in [0, 100] for completions")
        n = _int_field(body, "n_probs", 0, vmax) or 0
        return lp is not None or n > 0, (lp if lp is not None else n), bool(post)
    n = _int_field(body, "n_probs", 0, vmax) or 0
    return n > 0, n, bool(post)


def _job_from(body: Dict[str, Any], ids: List[int], default_max: int,
              vocab: Optional[int] = None, tok: Optional[Tokenizer] = None,
              stop_ids=(), api: str = "native") -> Job:
    """A request body -> Job.  Fields the server cannot honour are rejected (ValueError -> HTTP
    400) rather than ignored: ``n`` other than 1, a grammar / schema outside what
    grammar.py enforces, malformed probability requests."""
    from .grammar import GrammarState, grammar_from_request, matcher_for

    n_choices = body.get("n")
    if n_choices is not None and n_choices != 1:
        raise ValueError("n: only one choice per request is supported (n = 1)")
    stop = body.get("stop") or []
    if isinstance(stop, str):
        stop = [stop]
    n = body.get("n_predict", body.get("max_tokens", body.get("max_completion_tokens")))
    if n is None or int(n) < 0:
        n = default_max
    want, n_probs, post = _probs_request(body, api, vocab)
    src = grammar_from_request(body)
    gstate = None
    if src is not None:
        if tok is None:
            raise ValueError("grammar: this server has no tokenizer to constrain with")
        gstate = GrammarState(matcher_for(src), tok, stop_ids)
    return Job(ids=ids, max_new=int(n), params=SamplingParams.from_request(body, vocab),
               seed=None if body.get("seed") in (None, -1) else int(body["seed"]), stop=list(stop),
               cache_prompt=bool(body.get("cache_prompt", True)),
               ignore_eos=bool(body.get("ignore_eos", False)), grammar=gstate,
               n_probs=int(n_probs), want_probs=want, post_probs=post)


def _native_probs(entries: List[dict], post: bool) -> List[dict]:
    """llama-server's ``completion_probabilities`` items."""
    key, tkey = ("prob", "top_probs") if post else ("logprob", "top_logprobs")
    return [{"id": e["id"], "token": e["token"], "bytes": e["bytes"], key: e[key],
             tkey: [{"id": t["id"], "token": t["token"], "bytes": t["bytes"], key: t[key]}
                    for t in e["top"]]} for e in entries]


def _chat_logprobs(entries: List[dict]) -> Dict[str, Any]:
    """OpenAI chat ``choices[].logprobs``."""
    def lp(e):
        return e["logprob"] if "logprob" in e else (math.log(e["prob"]) if e["prob"] > 0
                                                     else -9999.0)
    return {"content": [{"token": e["token"], "logprob": lp(e), "bytes": e["bytes"],
                         "top_logprobs": [{"token": t["token"], "logprob": lp(t),
                                           "bytes": t["bytes"]} for t in e["top"]]}
                        for e in entries]}


def _completion_logprobs(entries: List[dict], offset: int = 0) -> Dict[str, Any]:
    """OpenAI (legacy) completions ``choices[].logprobs``."""
    def lp(e):
        return e["logprob"] if "logprob" in e else (math.log(e["prob"]) if e["prob"] > 0
                                                     else -9999.0)
    offs = []
    for e in entries:
        offs.append(offset)
        offset += len(e["token"])
    return {"tokens": [e["token"] for e in entries], "token_logprobs": [lp(e) for e in entries],
            "top_logprobs": [{t["token"]: lp(t) for t in e["top"]} for e in entries],
            "text_offset": offs}


class RequestTimeout(RuntimeError):
    pass


async def _events(job: Job, timeout: float, disconnected=None):
    """(kind, value) events of ``job`` as the scheduler produces them.  The scheduler wakes this
    coroutine with one ``call_soon_threadsafe`` per event loop and step (``Scheduler._wake``), so a
    waiting request holds no executor thread (polling through ``run_in_executor`` made
    token delivery queue behind idle connections).  After 0.5 s without an event
    ``disconnected()`` is polled: a client that went away while its job waits for a slot or
    between tokens is noticed and the job cancelled (``ConnectionAbortedError``); past
    ``timeout`` the job is cancelled and ``RequestTimeout`` raised."""
    deadline = time.perf_counter() + timeout
    loop = asyncio.get_running_loop()
    ev = asyncio.Event()
    job.waker = (loop, ev)                 # registered before the queue is looked at
    try:
        while True:
            try:
                kind, val = job.out.get_nowait()
            except queue.Empty:
                ev.clear()
                if not job.out.empty():
                    continue
                left = deadline - time.perf_counter()
                if left <= 0:
                    job.cancelled = True
                    raise RequestTimeout("request timed out")
                tick = loop.call_later(min(left, 0.5), ev.set)
                await ev.wait()
                tick.cancel()
                if job.out.empty() and disconnected is not None and await disconnected():
                    job.cancelled = True
                    raise ConnectionAbortedError("client disconnected")
                continue
            yield kind, val
            if kind in ("done", "error"):
                return
    finally:
        job.waker = None


async def _collect(job: Job, timeout: float, disconnected=None) -> Job:
    """The finished ``job`` (RuntimeError on its error); see ``_events``."""
    async for kind, val in _events(job, timeout, disconnected):
        if kind == "error":
            raise RuntimeError(val)
        if kind == "done":
            return val
    raise RuntimeError("job ended without a result")


async def _astream(job: Job, timeout: float, disconnected=None):
    """Events of ``job`` for a streaming response; a client that goes away (``disconnected()``,
    or the response generator closed) cancels the job, whose slot is freed at the next step."""
    finished = False
    try:
        async for kind, val in _events(job, timeout, disconnected):
            if kind == "error":
                raise RuntimeError(val)
            yield kind, val
            if kind == "done":
                finished = True
                return
    except ConnectionAbortedError:
        return
    finally:
        if not finished:
            job.cancelled = True


def _usage(job: Job) -> Dict[str, int]:
    return {"prompt_tokens": len(job.ids), "completion_tokens": len(job.gen),
            "total_tokens": len(job.ids) + len(job.gen)}


def _timings(job: Job) -> Dict[str, Any]:
    now = time.perf_counter()
    pred_ms = (now - job.t_first) * 1e3
    n = len(job.gen)
    n_prompt = len(job.ids) - job.n_cached
    return {"cache_n": job.n_cached, "prompt_n": n_prompt, "prompt_ms": round(job.t_prefill * 1e3, 3),
            "prompt_per_second": round(n_prompt / max(job.t_prefill, 1e-9), 2),
            "predicted_n": n, "predicted_ms": round(pred_ms, 3),
            "predicted_per_second": round(max(n - 1, 0) / max(pred_ms / 1e3, 1e-9), 2)}


def create_app(state: Dict[str, Any], request_timeout: float = 600.0):
    """``state``: {"scheduler": Scheduler | None, "tok": Tokenizer | None, "model": name}; the
    scheduler may be attached later (``/health`` answers 503 until then)."""
    from fastapi import FastAPI, HTTPException
    from fastapi.responses import JSONResponse, PlainTextResponse, StreamingResponse
    from starlette.concurrency import run_in_threadpool

    from .chat_template import TemplateError

    app = FastAPI(title="amdk8s llm server")

    def sched() -> Scheduler:
        s = state.get("scheduler")
        if s is None:
            raise HTTPException(503, "Loading model")
        return s

    def encode_prompt(p) -> List[int]:
        if isinstance(p, list) and all(isinstance(x, int) for x in p):
            return list(p)
        if isinstance(p, list):
            p = "".join(str(x) for x in p)
        return state["tok"].encode(str(p))

    async def aencode(p) -> List[int]:
        """BPE of a long prompt off the event loop (it would stall /health and every stream)."""
        return await run_in_threadpool(encode_prompt, p)

    def chat_prompt(body: Dict[str, Any]) -> str:
        msgs = body.get("messages") or []
        if not isinstance(msgs, list) or not msgs:
            raise HTTPException(400, "messages must be a non-empty list")
        tools = body.get("tools") or None
        try:
            return state["tok"].formatter.render(msgs, add_generation_prompt=True, tools=tools)
        except TemplateError as e:
            raise HTTPException(400, str(e))

    async def achat_ids(body: Dict[str, Any]) -> List[int]:
        def work():
            return state["tok"].encode(chat_prompt(body))
        return await run_in_threadpool(work)

    @app.get("/health")
    def health():
        if state.get("scheduler") is None:
            return JSONResponse({"error": {"code": 503, "message": "Loading model",
                                           "type": "unavailable_error"}}, status_code=503)
        return {"status": "ok"}

    @app.get("/v1/models")
    def models():
        return {"object": "list", "data": [{"id": state.get("model", "model"), "object": "model",
                                            "created": int(state.get("created", 0)),
                                            "owned_by": "amdk8s"}]}

    @app.post("/tokenize")
    def tokenize(body: Dict[str, Any]):
        return {"tokens": encode_prompt(body.get("content", ""))}

    @app.post("/detokenize")
    def detokenize(body: Dict[str, Any]):
        return {"content": state["tok"].decode(body.get("tokens", []))}

    def submit(body, ids, default_max, api="native"):
        s = sched()
        try:
            return s.submit(_job_from(body, ids, default_max, s.engine.cfg.vocab, state["tok"],
                                      s.stop_ids, api))
        except ValueError as e:
            raise HTTPException(400, str(e))

    async def prewarm(body: Dict[str, Any]) -> None:
        """A constrained request needs the vocabulary's byte trie (~2 s once for a 152k
        vocabulary): build it in the thread pool, not on the event loop or the GPU thread."""
        if any(body.get(k) for k in ("grammar", "json_schema", "response_format")):
            from .grammar import trie_for

            await run_in_threadpool(trie_for, state["tok"])

    async def wait(job: Job, request: Request) -> Job:
        try:
            return await _collect(job, request_timeout, request.is_disconnected)
        except RequestTimeout as e:
            raise HTTPException(504, str(e))
        except ConnectionAbortedError as e:
            raise HTTPException(499, str(e))
        except RuntimeError as e:
            raise HTTPException(500, str(e))

    @app.post("/completion")
    async def completion(body: Dict[str, Any], request: Request):
        s = sched()
        await prewarm(body)
        job = submit(body, await aencode(body.get("prompt", "")), s.engine.max_ctx)
        if body.get("stream"):
            async def gen():
                pend: List[dict] = []
                async for kind, val in _astream(job, request_timeout, request.is_disconnected):
                    if kind == "probs":
                        pend.append(val)
                        continue
                    if kind == "text":
                        d = {"content": val, "stop": False}
                    else:
                        d = {"content": "", "stop": True, "timings": _timings(val)}
                    if job.want_probs and pend:
                        d["completion_probabilities"] = _native_probs(pend, job.post_probs)
                        pend = []
                    yield "data: " + json.dumps(d) + "\n\n"
            return StreamingResponse(gen(), media_type="text/event-stream")
        job = await wait(job, request)
        out = {"content": job.text, "stop": True, "model": state.get("model"),
               "tokens_predicted": len(job.gen), "tokens_evaluated": len(job.ids),
               "tokens_cached": job.pos,
               "stopped_eos": job.finish == "stop" and job.gen[-1] in s.stop_ids,
               "stopped_limit": job.finish == "length",
               "stopped_word": (job.finish == "stop" and job.gen[-1] not in s.stop_ids
                                and job.grammar is None),
               "timings": _timings(job)}
        if job.want_probs:
            out["completion_probabilities"] = _native_probs(job.probs, job.post_probs)
        return out

    async def openai(body, ids, chat: bool, request: Request):
        s = sched()
        await prewarm(body)
        job = submit(body, ids, 16 if not chat else s.engine.max_ctx,
                     "chat" if chat else "completions")

        def lp_block(entries, offset=0):
            return _chat_logprobs(entries) if chat else _completion_logprobs(entries, offset)
        rid = ("chatcmpl-" if chat else "cmpl-") + uuid.uuid4().hex[:24]
        created = int(time.time())
        obj = "chat.completion" if chat else "text_completion"
        if body.get("stream"):
            async def gen():
                first = True
                pend: List[dict] = []
                sent = 0
                async for kind, val in _astream(job, request_timeout, request.is_disconnected):
                    if kind == "probs":
                        pend.append(val)
                        continue
                    if kind == "text":
                        if chat:
                            delta = {"content": val}
                            if first:
                                delta["role"] = "assistant"
                            ch = {"index": 0, "delta": delta, "finish_reason": None}
                        else:
                            ch = {"index": 0, "text": val, "finish_reason": None}
                        if job.want_probs:
                            ch["logprobs"] = lp_block(pend, sent)
                            sent += sum(len(e["token"]) for e in pend)
                            pend = []
                        first = False
                        yield "data: " + json.dumps({"id": rid, "object": obj + ".chunk" if chat
                                                     else obj, "created": created,
                                                     "model": state.get("model"),
                                                     "choices": [ch]}) + "\n\n"
                    else:     # the last chunk carries usage and llama-server's timings
                        ch = {"index": 0, "finish_reason": val.finish}
                        ch["delta" if chat else "text"] = {} if chat else ""
                        if job.want_probs and pend:
                            ch["logprobs"] = lp_block(pend, sent)
                        yield "data: " + json.dumps({"id": rid, "object": obj + ".chunk" if chat
                                                     else obj, "created": created,
                                                     "model": state.get("model"),
                                                     "choices": [ch], "usage": _usage(val),
                                                     "timings": _timings(val)}) + "\n\n"
                yield "data: [DONE]\n\n"
            return StreamingResponse(gen(), media_type="text/event-stream")
        job = await wait(job, request)
        choice = {"index": 0, "finish_reason": job.finish,
                  "logprobs": lp_block(job.probs) if job.want_probs else None}
        if chat:
            choice["message"] = {"role": "assistant", "content": job.text}
        else:
            choice["text"] = job.text
        return {"id": rid, "object": obj, "created": created, "model": state.get("model"),
                "choices": [choice],
                "usage": _usage(job),
                "timings": _timings(job)}

    @app.post("/v1/completions")
    async def v1_completions(body: Dict[str, Any], request: Request):
        return await openai(body, await aencode(body.get("prompt", "")), False, request)

    @app.post("/v1/chat/completions")
    async def v1_chat(body: Dict[str, Any], request: Request):
        sched()
        return await openai(body, await achat_ids(body), True, request)

    @app.post("/apply-template")
    def apply_template(body: Dict[str, Any]):
        """llama-server's endpoint: the prompt the chat template makes of ``messages``."""
        sched()
        return {"prompt": chat_prompt(body)}

    @app.get("/props")
    def props():
        s = sched()
        d = SamplingParams.from_request({})
        fmt = state["tok"].formatter
        return {"total_slots": s.parallel, "model_path": state.get("model"),
                "chat_template": fmt.source or "", "chat_template_source": fmt.kind,
                "default_generation_settings": {
                    "n_ctx": s.engine.max_ctx, "temperature": d.temperature, "top_k": d.top_k,
                    "top_p": d.top_p, "min_p": d.min_p, "repeat_penalty": d.repeat_penalty,
                    "repeat_last_n": d.repeat_last_n, "presence_penalty": d.presence_penalty,
                    "frequency_penalty": d.frequency_penalty, "cache_prompt": True}}

    @app.get("/slots")
    def slots():
        s = sched()
        return [{"id": i, "n_ctx": s.engine.max_ctx, "is_processing": i in s.active,
                 "n_cached": len(s.slot_tokens.get(i, []))} for i in range(s.parallel)]

    @app.get("/debug/iterations")
    def iterations(n: int = 2048):
        """The scheduler's last ``n`` loop iterations (perf_counter seconds, which is
        CLOCK_MONOTONIC: comparable across processes) and GC pauses — what a stalled stream
        waited on."""
        s = sched()
        keys = ("t", "admit_s", "prefill_s", "step_s", "wake_s", "prompt_tokens", "decoded")
        its = [dict(zip(keys, x)) for x in list(s.trace)[-max(1, n):]]
        gcs = [{"t": t, "s": d, "generation": g} for t, d, g in list(s.gc_pauses)]
        return {"iterations": its, "gc_pauses": gcs}

    @app.get("/metrics")
    def metrics():
        s = state.get("scheduler")
        m = dict(s.metrics) if s else {}
        lines = []
        for k, v in sorted(m.items()):
            name = f"llamacpp_amdk8s_{k}"
            lines += [f"# TYPE {name} {'counter' if k.endswith('_total') else 'gauge'}",
                      f"{name} {v}"]
        if s and m.get("decode_seconds_total"):
            tps = m["tokens_predicted_total"] / max(m["decode_seconds_total"] +
                                                    m["prefill_seconds_total"], 1e-9)
            lines += ["# TYPE llamacpp_amdk8s_predicted_tokens_seconds gauge",
                      f"llamacpp_amdk8s_predicted_tokens_seconds {tps:.3f}"]
        return PlainTextResponse("\n".join(lines) + "\n")

    return app


def build_engine(args) -> tuple:
    """Load a GGUF (``-m``) or build a synthetic model (``--synthetic tiny|7b``)."""
    device = "cuda" if torch.cuda.is_available() else "cpu"
    if args.model:
        from .synthetic import load

        eng, tok = load(args.model, device=device, max_ctx=args.ctx_size, slots=args.parallel)
        return eng, tok, os.path.basename(args.model)
    from .config import QWEN25_7B, tiny
    from .synthetic import write_synthetic_gguf, load
    import tempfile

    if args.synthetic == "7b":
        from .tokenizer import Tokenizer, synthetic_vocab
        from .weights import ModelWeights

        w = ModelWeights.random(QWEN25_7B, device=device)
        eng = Engine(w, max_ctx=args.ctx_size, slots=args.parallel)
        return eng, Tokenizer.from_gguf(synthetic_vocab(QWEN25_7B.vocab)), "qwen2.5-7b-synthetic"
    path = os.path.join(tempfile.mkdtemp(prefix="amdk8s-llm-"), "tiny.gguf")
    write_synthetic_gguf(path, tiny())
    eng, tok = load(path, device=device, max_ctx=args.ctx_size, slots=args.parallel)
    return eng, tok, "tiny-qwen2-synthetic"


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="llama-server-compatible API on the in-tree engine")
    ap.add_argument("-m", "--model", default=os.environ.get("MODEL_PATH"))
    ap.add_argument("--synthetic", choices=["tiny", "7b"], default="tiny",
                    help="random-weight model when no -m is given (offline)")
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=8080)
    ap.add_argument("-c", "--ctx-size", type=int, default=4096)
    ap.add_argument("-np", "--parallel", type=int, default=8,
                    help="KV-cache slots = sequences sharing one decode step (the engine steps "
                         "up to 8 tokens per pass over the weights)")
    ap.add_argument("-ub", "--ubatch-size", type=int, default=512,
                    help="prompt tokens per chunk while other sequences decode (llama-server -ub)")
    ap.add_argument("-b", "--batch-size", type=int, default=2048,
                    help="prompt tokens per chunk while nothing decodes (llama-server -b)")
    ap.add_argument("-ngl", "--n-gpu-layers", type=int, default=999, help="accepted; all layers run on the GPU")
    ap.add_argument("-t", "--threads", type=int, default=0, help="accepted; the GPU does the work")
    ap.add_argument("--no-prompt-batch", action="store_true",
                    help="prefill every prompt alone instead of batching the prompts admitted "
                         "together: a prompt's logits then never depend on concurrent traffic")
    ap.add_argument("-to", "--timeout", type=float, default=600.0,
                    help="seconds a request may wait for its result (then 504 and cancelled)")
    args = ap.parse_args(argv)
    import uvicorn

    state: Dict[str, Any] = {"scheduler": None, "tok": None, "model": "loading",
                             "created": time.time()}
    app = create_app(state, request_timeout=args.timeout)

    def load_bg():
        eng, tok, name = build_engine(args)
        if eng.gpu:
            eng.capture(range(1, min(args.parallel, eng.max_T) + 1))   # HIP graphs before ready
            eng.warmup()                                                # prompt path, first use
        state.update(tok=tok, model=name, scheduler=Scheduler(eng, tok, args.parallel,
                                                            ubatch=args.ubatch_size,
                                                            batch=args.batch_size,
                                                            prompt_batch=not args.no_prompt_batch))
        print(f"model {name} ready (ctx {eng.max_ctx}, parallel {args.parallel})", flush=True)

    threading.Thread(target=load_bg, daemon=True).start()
    uvicorn.run(app, host=args.host, port=args.port, log_level="info")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
