"""Common job engine: ReconcileJobs, expectations, work queues, manager."""
