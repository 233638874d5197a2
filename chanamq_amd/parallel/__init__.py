"""chanamq_amd.parallel"""
