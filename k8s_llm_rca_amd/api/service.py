"""In-process assistant service: the replacement for the OpenAI Assistants API.

The reference drives GPT-4 through ``client.beta.assistants/threads/runs``
(``common/openai_generic_assistant.py:16-133``).  This module keeps that
stateful model -- an *assistant* is (instructions, name, model), a *thread* is
an append-only conversation, a *run* generates one assistant reply
conditioned on the whole thread -- but executes runs on a local backend:

* :class:`~k8s_llm_rca_amd.engine.backend.EngineBackend` - the MI355X LLM
  engine (continuous batching across every active run, per-thread paged-KV
  prefix reuse, grammar-constrained decoding);
* :class:`ScriptedBackend` - a deterministic responder for tests.

Runs complete by event notification, not by the reference's
``sleep(5*i)`` polling (``openai_generic_assistant.py:92-115``).
Result objects mirror the OpenAI SDK shapes the reference reads:
``messages.data[0].content[0].text.value``, ``run.status``, ``run.usage``,
``run.created_at`` / ``run.completed_at``.
"""
from __future__ import annotations

import itertools
import logging
import threading
import time
import uuid
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional

log = logging.getLogger(__name__)

TERMINAL = ("completed", "failed", "cancelled", "expired")


def _id(prefix: str) -> str:
    return f"{prefix}_{uuid.uuid4().hex[:24]}"


@dataclass
class Text:
    value: str
    annotations: list = field(default_factory=list)


@dataclass
class TextContent:
    text: Text
    type: str = "text"


@dataclass
class Message:
    id: str
    thread_id: str
    role: str
    content: List[TextContent]
    created_at: float
    assistant_id: Optional[str] = None
    run_id: Optional[str] = None
    object: str = "thread.message"

    @property
    def text(self) -> str:
        return self.content[0].text.value


@dataclass
class MessageList:
    data: List[Message]
    has_more: bool = False
    object: str = "list"

    def __iter__(self):
        return iter(self.data)

    def __len__(self):
        return len(self.data)


@dataclass
class Assistant:
    id: str
    name: str
    instructions: str
    model: str
    created_at: float
    object: str = "assistant"


@dataclass
class Thread:
    id: str
    created_at: float
    object: str = "thread"


@dataclass
class Run:
    id: str
    thread_id: str
    assistant_id: str
    status: str
    created_at: float
    instructions: Optional[str] = None
    model: str = ""
    started_at: Optional[float] = None
    completed_at: Optional[float] = None
    failed_at: Optional[float] = None
    last_error: Optional[str] = None
    usage: Optional[Dict[str, int]] = None
    object: str = "thread.run"


class ThreadState:
    """Server-side thread: messages + backend cache handle (e.g. KV blocks)."""

    def __init__(self, thread: Thread):
        self.thread = thread
        self.messages: List[Message] = []
        self.lock = threading.Lock()
        self.active_run: Optional[str] = None
        self.backend_state: Any = None  # owned by the backend (token ids, KV sequence, ...)


class RunState:
    def __init__(self, run: Run, thread: ThreadState, assistant: Assistant, response_format: Any,
                 max_tokens: Optional[int], sampling: Optional[dict]):
        self.run = run
        self.thread = thread
        self.assistant = assistant
        self.response_format = response_format
        self.max_tokens = max_tokens
        self.sampling = sampling or {}
        self.done = threading.Event()
        self.reply: Optional[str] = None
        self.metrics: Dict[str, float] = {}


class AssistantService:
    def __init__(self, backend: "Backend"):
        self.backend = backend
        self.assistants: Dict[str, Assistant] = {}
        self.threads: Dict[str, ThreadState] = {}
        self.runs: Dict[str, RunState] = {}
        self._runs_by_thread: Dict[str, List[str]] = {}
        self._lock = threading.Lock()
        self.closed = False
        backend.attach(self)

    def close(self) -> None:
        """Shut down: active runs are cancelled and every later run fails at
        once (callers' repair loops then end quickly instead of waiting)."""
        self.closed = True
        with self._lock:
            active = [r for r in self.runs.values() if not r.done.is_set()]
        for rs in active:
            self.cancel_run(rs.run.id)
        if active:  # one line for the shutdown, not one warning per cut-short run
            log.info("service closed: %d active run(s) cancelled", len(active))

    # ------------------------------------------------------------ assistants
    def create_assistant(self, instructions: str, name: str, model: str) -> Assistant:
        a = Assistant(_id("asst"), name, instructions, model, time.time())
        with self._lock:
            self.assistants[a.id] = a
        return a

    def retrieve_assistant(self, assistant_id: str) -> Assistant:
        with self._lock:
            a = self.assistants.get(assistant_id)
        if a is None:
            raise KeyError(f"No assistant found with id '{assistant_id}'")
        return a

    # --------------------------------------------------------------- threads
    def create_thread(self) -> Thread:
        t = Thread(_id("thread"), time.time())
        with self._lock:
            self.threads[t.id] = ThreadState(t)
            self._runs_by_thread[t.id] = []
        return t

    def retrieve_thread(self, thread_id: str) -> Thread:
        return self._thread(thread_id).thread

    def _thread(self, thread_id: str) -> ThreadState:
        with self._lock:
            ts = self.threads.get(thread_id)
        if ts is None:
            raise KeyError(f"No thread found with id '{thread_id}'")
        return ts

    def delete_thread(self, thread_id: str) -> None:
        ts = self._thread(thread_id)
        self.backend.release_thread(ts)
        with self._lock:
            self.threads.pop(thread_id, None)

    def add_message(self, thread_id: str, content: str, role: str = "user") -> Message:
        ts = self._thread(thread_id)
        with ts.lock:
            if ts.active_run is not None:
                raise RuntimeError(f"Can't add messages to {thread_id} while a run {ts.active_run} is active.")
            m = Message(_id("msg"), thread_id, role, [TextContent(Text(content))], time.time())
            ts.messages.append(m)
        return m

    def list_messages(self, thread_id: str, limit: int = 20, order: str = "desc") -> MessageList:
        ts = self._thread(thread_id)
        with ts.lock:
            msgs = list(ts.messages)
        if order == "desc":
            msgs = msgs[::-1]
        return MessageList(msgs[:limit], has_more=len(msgs) > limit)

    # --------------------------------------------------------- persistence
    def export_state(self) -> dict:
        """Assistants + threads + messages as plain JSON (resume across processes,
        the reference's retrieve_assistant / retrieve_thread, openai_generic_assistant.py:25-35)."""
        with self._lock:
            asst = [vars(a).copy() for a in self.assistants.values()]
            threads = []
            for ts in self.threads.values():
                with ts.lock:
                    threads.append({"id": ts.thread.id, "created_at": ts.thread.created_at,
                                    "messages": [{"id": m.id, "role": m.role, "text": m.text,
                                                  "created_at": m.created_at, "assistant_id": m.assistant_id,
                                                  "run_id": m.run_id} for m in ts.messages]})
        return {"assistants": asst, "threads": threads}

    def import_state(self, state: dict) -> None:
        with self._lock:
            for a in state.get("assistants", []):
                self.assistants[a["id"]] = Assistant(**a)
            for t in state.get("threads", []):
                ts = ThreadState(Thread(t["id"], t["created_at"]))
                for m in t["messages"]:
                    ts.messages.append(Message(m["id"], t["id"], m["role"], [TextContent(Text(m["text"]))],
                                               m["created_at"], m.get("assistant_id"), m.get("run_id")))
                self.threads[t["id"]] = ts
                self._runs_by_thread.setdefault(t["id"], [])

    # ------------------------------------------------------------------ runs
    def create_run(self, thread_id: str, assistant_id: str, instructions: Optional[str] = None,
                   response_format: Any = None, max_tokens: Optional[int] = None,
                   sampling: Optional[dict] = None) -> Run:
        ts = self._thread(thread_id)
        a = self.retrieve_assistant(assistant_id)
        r = Run(_id("run"), thread_id, assistant_id, "queued", time.time(),
                instructions=instructions, model=a.model)
        rs = RunState(r, ts, a, response_format, max_tokens, sampling)
        with ts.lock:
            if ts.active_run is not None:
                raise RuntimeError(f"Thread {thread_id} already has an active run {ts.active_run}.")
            ts.active_run = r.id
        with self._lock:
            self.runs[r.id] = rs
            self._runs_by_thread[thread_id].append(r.id)
        if self.closed:
            self._finish(rs, None, "failed", error="service closed")
            return r
        self.backend.submit(rs)
        return r

    def retrieve_run(self, thread_id: str, run_id: str) -> Run:
        with self._lock:
            rs = self.runs.get(run_id)
        if rs is None or rs.run.thread_id != thread_id:
            raise KeyError(f"No run found with id '{run_id}'")
        return rs.run

    def list_runs(self, thread_id: str, limit: int = 20, order: str = "desc") -> List[Run]:
        with self._lock:
            ids = list(self._runs_by_thread.get(thread_id, []))
        runs = [self.runs[i].run for i in ids]
        if order == "desc":
            runs = runs[::-1]
        return runs[:limit]

    def wait_run(self, run_id: str, timeout: Optional[float] = None) -> Run:
        with self._lock:
            rs = self.runs[run_id]
        if not rs.done.wait(timeout):
            self.cancel_run(run_id, status="expired")
        return rs.run

    def cancel_run(self, run_id: str, status: str = "cancelled") -> None:
        with self._lock:
            rs = self.runs[run_id]
        if rs.done.is_set():
            return
        self.backend.cancel(rs)
        self._finish(rs, None, status, error=status)

    # ----------------------------------------------------- backend callbacks
    def run_started(self, rs: RunState) -> None:
        rs.run.status = "in_progress"
        rs.run.started_at = time.time()

    def run_completed(self, rs: RunState, reply: str, prompt_tokens: int, completion_tokens: int,
                      metrics: Optional[Dict[str, float]] = None) -> None:
        rs.run.usage = {"prompt_tokens": int(prompt_tokens), "completion_tokens": int(completion_tokens),
                        "total_tokens": int(prompt_tokens + completion_tokens)}
        if metrics:
            rs.metrics.update(metrics)
        self._finish(rs, reply, "completed")

    def run_failed(self, rs: RunState, error: str) -> None:
        self._finish(rs, None, "failed", error=error)

    def _finish(self, rs: RunState, reply: Optional[str], status: str, error: Optional[str] = None) -> None:
        ts = rs.thread
        with ts.lock:
            if rs.done.is_set():
                return
            now = time.time()
            if reply is not None:
                ts.messages.append(Message(_id("msg"), ts.thread.id, "assistant", [TextContent(Text(reply))],
                                           now, assistant_id=rs.assistant.id, run_id=rs.run.id))
            rs.reply = reply
            rs.run.status = status
            if status == "completed":
                rs.run.completed_at = now
            else:
                rs.run.failed_at = now
                rs.run.last_error = error
            if ts.active_run == rs.run.id:
                ts.active_run = None
            rs.done.set()


class Backend:
    """Interface implemented by the LLM engine backend and the scripted backend."""

    def attach(self, service: AssistantService) -> None:
        self.service = service

    def submit(self, rs: RunState) -> None:
        raise NotImplementedError

    def cancel(self, rs: RunState) -> None:
        pass

    def release_thread(self, ts: ThreadState) -> None:
        pass


def _approx_tokens(text: str) -> int:
    return max(1, (len(text) + 3) // 4)


class ScriptedBackend(Backend):
    """Deterministic responder: ``responder(run_state) -> str``, executed inline.

    Used by tests to exercise pipeline control flow (including malformed
    replies that drive the repair loops) without a model.
    """

    def __init__(self, responder: Callable[[RunState], str], tokenizer=None):
        self.responder = responder
        self.tokenizer = tokenizer
        self.calls = 0

    def _count(self, text: str) -> int:
        if self.tokenizer is not None:
            return len(self.tokenizer.encode(text))
        return _approx_tokens(text)

    def submit(self, rs: RunState) -> None:
        self.calls += 1
        self.service.run_started(rs)
        try:
            reply = self.responder(rs)
        except Exception as e:  # a failing responder == a failed run
            self.service.run_failed(rs, repr(e))
            return
        if reply is None:
            self.service.run_failed(rs, "responder returned None")
            return
        sys_text = rs.run.instructions or rs.assistant.instructions
        prompt = sys_text + "".join(m.text for m in rs.thread.messages)
        self.service.run_completed(rs, reply, self._count(prompt), self._count(reply))


_default_service: Optional[AssistantService] = None
_default_lock = threading.Lock()


def set_default_service(service: Optional[AssistantService]) -> None:
    global _default_service
    with _default_lock:
        _default_service = service


def get_default_service() -> AssistantService:
    with _default_lock:
        if _default_service is None:
            raise RuntimeError("no AssistantService configured: call "
                               "k8s_llm_rca_amd.api.service.set_default_service(...) first")
        return _default_service
