"""``GenericAssistant`` -- client object with the reference's assistant API.

Method-for-method equivalent of ``OpenAIGenericAssistant``
(``common/openai_generic_assistant.py:10-135``):

=========================  ===============================================
reference                  here
=========================  ===============================================
``create_assistant``       creates an assistant on the in-process service
``retrieve_assistant``     looks one up (resume, ``:25-27``)
``create_thread``          new append-only conversation
``retrieve_thread``        resume a thread (``:33-35``)
``add_message``            append a *user* message, no generation (``:37-43``)
``run_assistant``          start a run over the whole thread (``:45-51``)
``get_run_status``         current run object (``:53-58``)
``display_response`` etc.  message readers (``:60-90``)
``wait_get_last_k_message`` block until the run finishes -- event-driven,
                           no ``sleep(5*i)`` quantum (``:92-115``); returns
                           ``None`` for cancelled / failed / expired runs
``get_token_usage``        sum ``usage`` of runs created *and* completed in
                           ``[tmin, tmax)`` (``:117-135``)
=========================  ===============================================

``run_assistant`` additionally accepts ``response_format`` (a grammar from
:mod:`k8s_llm_rca_amd.engine.structured`), ``max_tokens`` and sampling
overrides; omitted, behaviour matches the reference.
"""
from __future__ import annotations

import logging
from typing import Any, Dict, Optional

from .service import AssistantService, MessageList, Run, get_default_service

log = logging.getLogger(__name__)

DEFAULT_MODEL = "llama3-8b"
# the reference waits at most sum(5*i for i in 1..120) seconds (openai_generic_assistant.py:94-97)
DEFAULT_RUN_TIMEOUT_S = float(sum(5 * i for i in range(1, 121)))


class GenericAssistant:
    def __init__(self, service: Optional[AssistantService] = None):
        self.service = service or get_default_service()
        self.assistant = None
        self.thread = None
        self.run = None
        self.message = None

    def create_assistant(self, instructions: str, name: str, model: str = DEFAULT_MODEL):
        self.assistant = self.service.create_assistant(instructions, name, model)

    def retrieve_assistant(self, assistant_id: str):
        self.assistant = self.service.retrieve_assistant(assistant_id)

    def create_thread(self):
        self.thread = self.service.create_thread()

    def retrieve_thread(self, thread_id: str):
        self.thread = self.service.retrieve_thread(thread_id)

    def add_message(self, content: str):
        self.message = self.service.add_message(self.thread.id, content, role="user")

    def run_assistant(self, instructions: Optional[str] = None, response_format: Any = None,
                      max_tokens: Optional[int] = None, sampling: Optional[Dict[str, Any]] = None):
        self.run = self.service.create_run(self.thread.id, self.assistant.id, instructions=instructions,
                                           response_format=response_format, max_tokens=max_tokens,
                                           sampling=sampling)

    def get_run_status(self) -> Run:
        return self.service.retrieve_run(self.thread.id, self.run.id)

    def display_response(self):
        messages = self.service.list_messages(self.thread.id, limit=1)
        print(messages.data[0])

    def get_last_message(self) -> MessageList:
        return self.service.list_messages(self.thread.id, limit=1)

    def get_all_message(self) -> MessageList:
        return self.service.list_messages(self.thread.id)

    def get_last_k_message(self, num: int) -> MessageList:
        return self.service.list_messages(self.thread.id, limit=num)

    def wait_get_last_k_message(self, num: int = 1, timeout: float = DEFAULT_RUN_TIMEOUT_S):
        run = self.service.wait_run(self.run.id, timeout)
        if run.status == "completed":
            return self.get_last_k_message(num)
        if not self.service.closed:  # runs cut short by a shutdown are summarised by close()
            log.warning("run %s %s", run.id, run.status)
        return None

    def get_token_usage(self, tmin: float, tmax: float, limit: int = 20) -> Dict[str, int]:
        usage = {"prompt_tokens": 0, "completion_tokens": 0, "total_tokens": 0}
        for run in self.service.list_runs(self.thread.id, limit=limit, order="desc"):
            if run.created_at is None or run.completed_at is None or run.usage is None:
                continue
            if tmin <= run.created_at < tmax and tmin <= run.completed_at < tmax:
                for k in usage:
                    usage[k] += run.usage[k]
        return usage


# name used by the reference (common/openai_generic_assistant.py:10)
OpenAIGenericAssistant = GenericAssistant
