"""avenir_amd.models"""
