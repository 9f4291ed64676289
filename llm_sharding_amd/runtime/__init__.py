"""Per-stage execution engine (StageEngine) and hipGraph-captured decode steps."""
