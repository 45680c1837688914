"""@calTimes wall-clock decorator (reference utils/wrapper.py:12-32)."""
import functools
import time


def calTimes(logger, msg: str):
    def dector(func):
        @functools.wraps(func)
        def wrapper(*arg, **kwarg):
            t0 = time.time()
            res = func(*arg, **kwarg)
            logger.info((msg + "，" if msg else "") + "耗时：%.2f s" % (time.time() - t0))
            return res
        return wrapper
    return dector
