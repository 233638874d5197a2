"""chanamq_amd.utils"""
