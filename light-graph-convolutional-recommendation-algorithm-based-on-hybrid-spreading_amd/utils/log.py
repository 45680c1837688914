"""Console logger with the reference's interface (reference utils/log.py:14-97)."""
import logging

logger = logging.getLogger("lgcnhs")
if not logger.handlers:
    _h = logging.StreamHandler()
    _h.setFormatter(logging.Formatter("%(asctime)s - %(name)s - %(levelname)s - %(message)s"))
    logger.addHandler(_h)
    logger.setLevel(logging.INFO)
Logger = logging.Logger
