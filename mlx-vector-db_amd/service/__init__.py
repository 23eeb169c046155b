"""Host side of the MI355X vector-search core, laid out like the reference's
``service`` package (reference service/__init__.py) so that
``from service.optimized_vector_store import MLXVectorStore`` keeps working."""
