"""chanamq_amd.models"""
