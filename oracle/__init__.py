"""Test infrastructure only: the CPU restatement (oracle) of aws-checksums' arithmetic."""
