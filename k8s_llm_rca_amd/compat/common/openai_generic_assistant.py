"""``common/openai_generic_assistant.py`` path: :class:`OpenAIGenericAssistant`."""
from k8s_llm_rca_amd.api.assistant import GenericAssistant


class OpenAIGenericAssistant(GenericAssistant):
    """No API key and no ``OpenAI()`` client: runs execute on the in-process
    service (``openai_generic_assistant.py:11-14``)."""


__all__ = ["OpenAIGenericAssistant"]
