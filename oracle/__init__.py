"""ORACLE TEST INFRASTRUCTURE (never imported by the product path)."""
