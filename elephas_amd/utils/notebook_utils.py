"""reference elephas/utils/notebook_utils.py:1-9"""


def is_running_in_notebook() -> bool:
    try:
        cfg = get_ipython().config  # noqa: F821
        return "IPKernelApp" in cfg
    except NameError:
        return False
