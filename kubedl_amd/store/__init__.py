"""Local API-server stand-in: object store, watch bus, event recorder."""
from kubedl_amd.store.store import (ADDED, DELETED, MODIFIED, AlreadyExists, Conflict,  # noqa: F401
                                    NotFound, Store, match_labels, obj_key)
from kubedl_amd.store.events import NORMAL, WARNING, EventRecorder  # noqa: F401
