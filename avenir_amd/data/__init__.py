"""avenir_amd.data"""
