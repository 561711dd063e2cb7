"""Job/pod/event persistence (``controllers/persist`` + ``pkg/storage``)."""
from kubedl_amd.persist.backends import (EventStorageBackend, JSONLEventBackend, ObjectStorageBackend,  # noqa: F401
                                         Query, SQLiteEventBackend, SQLiteObjectBackend,
                                         new_event_backend, new_object_backend)
