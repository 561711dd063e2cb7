"""Job/pod/event persistence (``controllers/persist`` + ``pkg/storage``)."""
from kubedl_amd.persist.backends import (EventStorageBackend, JSONLEventBackend, ObjectStorageBackend,  # noqa: F401
                                         Query, SQLiteEventBackend, SQLiteObjectBackend,
                                         new_event_backend, new_object_backend)
from kubedl_amd.persist import remote  # noqa: F401,E402  (registers mysql / aliyun-sls)
