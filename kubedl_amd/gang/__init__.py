"""Gang scheduling: ``GangScheduler`` interface + registry + the local
all-or-nothing MI355X GPU allocator (``pkg/gang_schedule``)."""
from kubedl_amd.gang.interface import GangScheduler, get, names, register  # noqa: F401
from kubedl_amd.gang.allocator import GPUAllocator, GPUInventory, detect_gpus  # noqa: F401
from kubedl_amd.gang.local import LocalGangScheduler  # noqa: F401
