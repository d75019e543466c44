"""Workloads the operator schedules onto MI355X: validator, GEMM benchmark, SD1.5 service, LLM."""
