"""Drop-in import name of the reference package (`import cnmf`, /root/reference/cnmf/__init__.py,
which is empty upstream): re-exports the MI355X implementation from `cnmf_amd`."""
from cnmf_amd import *  # noqa: F401,F403
from cnmf_amd import __all__, __version__  # noqa: F401
