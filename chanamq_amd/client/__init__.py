"""chanamq_amd.client"""
