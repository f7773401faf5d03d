"""``openai`` client surface over the in-process assistant service.

Only what the reference touches (``common/openai_generic_assistant.py:4-133``,
``test_token.py``): ``openai.api_key``; ``OpenAI()`` with
``beta.assistants.create/retrieve``, ``beta.threads.create/retrieve``,
``beta.threads.messages.create/list`` and ``beta.threads.runs.create/
retrieve/list``.  Every call goes to the default
:class:`~k8s_llm_rca_amd.api.service.AssistantService` (``set_default_service``:
the MI355X engine backend, or a scripted one in tests) instead of HTTPS; the
returned objects carry the SDK's attribute shapes (``messages.data[0].content
[0].text.value``, ``run.status``, ``run.usage['total_tokens']``,
``run.created_at``), so unchanged reference code runs.  No key is needed.
"""
from __future__ import annotations

from typing import Any, Optional

from k8s_llm_rca_amd.api.service import AssistantService, get_default_service

api_key: Optional[str] = None

__all__ = ["OpenAI", "api_key"]


class _Assistants:
    def __init__(self, svc: AssistantService):
        self._svc = svc

    def create(self, instructions: str = "", name: str = "", model: str = "gpt-4", **kw):
        return self._svc.create_assistant(instructions, name, model)

    def retrieve(self, assistant_id: str):
        return self._svc.retrieve_assistant(assistant_id)


class _Messages:
    def __init__(self, svc: AssistantService):
        self._svc = svc

    def create(self, thread_id: str, role: str = "user", content: str = "", **kw):
        return self._svc.add_message(thread_id, content, role=role)

    def list(self, thread_id: str, limit: int = 20, order: str = "desc", **kw):
        return self._svc.list_messages(thread_id, limit=limit, order=order)


class _Runs:
    def __init__(self, svc: AssistantService):
        self._svc = svc

    def create(self, thread_id: str, assistant_id: str, instructions: Optional[str] = None, **kw):
        return self._svc.create_run(thread_id, assistant_id, instructions=instructions,
                                    response_format=kw.get("response_format"), max_tokens=kw.get("max_tokens"))

    def retrieve(self, run_id: str = None, thread_id: str = None, **kw):
        return self._svc.retrieve_run(thread_id, run_id)

    def list(self, thread_id: str, order: str = "desc", limit: int = 20, **kw):
        return self._svc.list_runs(thread_id, limit=limit, order=order)

    def cancel(self, run_id: str = None, thread_id: str = None, **kw):
        self._svc.cancel_run(run_id)
        return self._svc.retrieve_run(thread_id, run_id)


class _Threads:
    def __init__(self, svc: AssistantService):
        self._svc = svc
        self.messages = _Messages(svc)
        self.runs = _Runs(svc)

    def create(self, **kw):
        return self._svc.create_thread()

    def retrieve(self, thread_id: str):
        return self._svc.retrieve_thread(thread_id)


class _Beta:
    def __init__(self, svc: AssistantService):
        self.assistants = _Assistants(svc)
        self.threads = _Threads(svc)


class OpenAI:
    """``OpenAI(api_key=None, service=None)``: ``service`` defaults to the
    process-wide default service at construction time."""

    def __init__(self, api_key: Optional[str] = None, service: Optional[AssistantService] = None, **kw: Any):
        self.service = service or get_default_service()
        self.beta = _Beta(self.service)
