"""Model loading (reference: src/awq_quantizer/model_loading/__init__.py).

load_model_from_hub() keeps the reference's behaviour of trying the Hub first and
falling back to treating the id as a local path (reference __init__.py:89-115); a local
directory or file is used directly without touching the network."""
import os
from typing import Optional

from ..utils.logger import get_logger
from .safetensors_loader import SafetensorsLoader, TensorInfo

__all__ = ["SafetensorsLoader", "TensorInfo", "load_model_from_hub", "load_model_from_path"]


def load_model_from_path(model_path: str, logger_name: str = "model_loading", logger_level: str = "INFO",
                         logger_to_file: bool = False, logger_file_path: Optional[str] = None,
                         verify_files: bool = True) -> SafetensorsLoader:
    return SafetensorsLoader(model_path=model_path, from_hub=False, logger_name=logger_name,
                             logger_level=logger_level, logger_to_file=logger_to_file,
                             logger_file_path=logger_file_path, resume_download=False, force_download=False)


def load_model_from_hub(model_id: str, revision: str = "main", token: Optional[str] = None,
                        logger_name: str = "model_loading", logger_level: str = "INFO",
                        logger_to_file: bool = False, logger_file_path: Optional[str] = None,
                        resume_download: bool = True, force_download: bool = False,
                        verify_downloads: bool = True) -> SafetensorsLoader:
    logger = get_logger(name=logger_name, level=logger_level, to_file=logger_to_file, file_path=logger_file_path)
    local_dir = model_id if os.path.exists(model_id) else None
    if local_dir is None:
        try:
            from huggingface_hub import snapshot_download
            local_dir = snapshot_download(repo_id=model_id, revision=revision, token=token,
                                          force_download=force_download)
            logger.info(f"Successfully downloaded model snapshot to {local_dir}")
        except Exception as e:  # noqa: BLE001 — offline or unknown id: fall back to a path
            logger.warning(f"Failed to download model snapshot: {e}")
            local_dir = model_id
    return SafetensorsLoader(model_path=local_dir, from_hub=False, revision=revision, token=token,
                             logger_name=logger_name, logger_level=logger_level, logger_to_file=logger_to_file,
                             logger_file_path=logger_file_path, resume_download=resume_download,
                             force_download=force_download)
