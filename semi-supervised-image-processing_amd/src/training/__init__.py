"""Training pipelines (mirror of the reference's src/training/)."""
