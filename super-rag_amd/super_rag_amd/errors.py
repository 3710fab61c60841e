"""Error types of the embed / rerank services (super_rag/llm/llm_error_types.py:13-299).

Inside a super_rag deployment the reference's own classes are re-exported, so callers that catch
``EmbeddingError`` / ``RerankError`` (nodeflow/runners/vector_search.py:95-105,
nodeflow/runners/rerank.py:90-103) keep working unchanged.  Standalone, the same hierarchy,
messages and ``details`` are defined here.
"""
from __future__ import annotations

from typing import Any, Dict, Optional

try:  # pragma: no cover - exercised only inside a super_rag deployment
    from super_rag.llm.llm_error_types import (  # type: ignore
        BatchProcessingError,
        EmbeddingError,
        EmptyTextError,
        InvalidConfigurationError,
        InvalidDocumentError,
        LLMError,
        ModelNotFoundError,
        ProviderNotFoundError,
        RerankError,
        TooManyDocumentsError,
    )
    HOST_ERRORS = True
except Exception:  # noqa: BLE001
    HOST_ERRORS = False

    class LLMError(Exception):
        def __init__(self, message: str, details: Optional[Dict[str, Any]] = None):
            super().__init__(message)
            self.message = message
            self.details = details or {}

        def __str__(self) -> str:
            if self.details:
                return f"{self.message} (Details: {self.details})"
            return self.message

    class LLMConfigurationError(LLMError):
        pass

    class ProviderNotFoundError(LLMConfigurationError):
        def __init__(self, provider_name: str, service_type: str = "LLM"):
            super().__init__(f"{service_type} provider '{provider_name}' not found or not configured",
                             {"provider_name": provider_name, "service_type": service_type})
            self.provider_name = provider_name
            self.service_type = service_type

    class ModelNotFoundError(LLMConfigurationError):
        def __init__(self, model_name: str, provider_name: str = None, service_type: str = "LLM"):
            message = f"{service_type} model '{model_name}' not found"
            if provider_name:
                message += f" for provider '{provider_name}'"
            super().__init__(message, {"model_name": model_name, "provider_name": provider_name,
                                       "service_type": service_type})
            self.model_name = model_name
            self.provider_name = provider_name
            self.service_type = service_type

    class InvalidConfigurationError(LLMConfigurationError):
        def __init__(self, config_field: str, config_value: Any = None,
                     reason: str = "Invalid configuration"):
            super().__init__(f"Invalid configuration for '{config_field}': {reason}",
                             {"config_field": config_field, "config_value": config_value,
                              "reason": reason})
            self.config_field = config_field
            self.config_value = config_value
            self.reason = reason

    class EmbeddingError(LLMError):
        pass

    class EmptyTextError(EmbeddingError):
        def __init__(self, text_count: int = 1):
            message = "Cannot embed empty text"
            if text_count > 1:
                message += f" (found {text_count} empty texts)"
            super().__init__(message, {"text_count": text_count})
            self.text_count = text_count

    class BatchProcessingError(EmbeddingError):
        def __init__(self, batch_size: int, failed_indices: list = None,
                     reason: str = "Batch processing failed"):
            details = {"batch_size": batch_size, "reason": reason}
            if failed_indices:
                details["failed_indices"] = failed_indices
            super().__init__(f"Batch processing error (batch size: {batch_size}): {reason}", details)
            self.batch_size = batch_size
            self.failed_indices = failed_indices or []
            self.reason = reason

    class RerankError(LLMError):
        pass

    class InvalidDocumentError(RerankError):
        def __init__(self, reason: str = "Invalid document format", document_count: int = None):
            message = f"Invalid documents for reranking: {reason}"
            if document_count is not None:
                message += f" (document count: {document_count})"
            super().__init__(message, {"reason": reason, "document_count": document_count})
            self.reason = reason
            self.document_count = document_count

    class TooManyDocumentsError(RerankError):
        def __init__(self, document_count: Optional[int] = None, max_documents: Optional[int] = None,
                     model_name: str = None):
            if document_count is not None and max_documents is not None:
                message = (f"Too many documents for reranking: {document_count} exceeds maximum "
                           f"{max_documents}")
            else:
                message = "Too many documents for reranking: document count exceeds model's limit"
            if model_name:
                message += f" for model '{model_name}'"
            super().__init__(message, {"document_count": document_count,
                                       "max_documents": max_documents, "model_name": model_name})
            self.document_count = document_count
            self.max_documents = max_documents
            self.model_name = model_name
