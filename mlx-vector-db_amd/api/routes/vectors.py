"""The reference's /vectors routes over the MI355X store.

Same paths, request bodies, response shapes and score formatting as
/root/reference/api/routes/vectors.py, so its SDKs (sdk/python/mlx_vector_client.py:346-404)
and HTTP scripts work unchanged:

  POST /vectors/add           {user_id, model_id, vectors, metadata}       (:163-207)
  POST /vectors/query         {user_id, model_id, query, k, filter_metadata} (:211-270)
  POST /vectors/batch_query   {user_id, model_id, queries, k}              (:272-330)
  GET  /vectors/count, /vectors/stats, /vectors/health                     (:332-388)

Differences, on purpose:
  * /batch_query works: the reference calls a ``store.batch_query`` that does not exist
    and always answers 500 (:291, :328-330); here the store's batched device search runs
    (service/optimized_vector_store.py ``batch_query``, which returns distances because
    this route scores cosine as ``max(0, 1 - dist)``, :300-306).
  * Stores are created lazily per (user, model) as in ``VectorStoreManager.get_store``
    (:48-71), under ``$VECTOR_STORE_BASE`` (default the reference's
    ``~/.team_mind_data/vector_stores``); the store config (metric, devices) comes from a
    factory the app may replace.

Scores (S12, :236-258): cosine ``similarity = raw, distance = 1 - raw``; euclidean
``distance = raw, similarity = 1 / (1 + distance)``; each result has ``rank`` and no
``index``.  Every store call runs on a 4-thread executor, like the reference (:43).
"""
from __future__ import annotations

import asyncio
import logging
import os
import secrets
import threading
import time
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path
from typing import Any, Callable, Dict, List, Optional

from fastapi import APIRouter, Depends, HTTPException, Security
from fastapi.security import HTTPAuthorizationCredentials, HTTPBearer
from pydantic import BaseModel, Field, model_validator

from service.optimized_vector_store import MLXVectorStore, MLXVectorStoreConfig

logger = logging.getLogger(__name__)


# ---- request / response models (service/models.py:34-61, api/routes/vectors.py:147-161) ----
class VectorAddRequest(BaseModel):
    user_id: str
    model_id: str
    vectors: List[List[float]] = Field(..., description="List of vectors to add")
    metadata: List[Dict[str, Any]] = Field(..., description="Metadata for each vector")

    @model_validator(mode="after")
    def validate_same_length(self):
        if len(self.vectors) != len(self.metadata):
            raise ValueError("Vectors and metadata must have the same length")
        return self


class VectorQuery(BaseModel):
    user_id: str
    model_id: str
    query: List[float] = Field(..., description="Query vector")
    k: int = Field(default=10, ge=1, le=1000)
    filter_metadata: Optional[Dict[str, Any]] = Field(default=None, description="Metadata filter")


class BatchQueryRequest(BaseModel):
    user_id: str
    model_id: str
    queries: List[List[float]]
    k: int = 10


class VectorAddResponse(BaseModel):
    success: bool
    vectors_added: int
    total_vectors: int
    processing_time_ms: float


class VectorQueryResponse(BaseModel):
    results: List[Dict[str, Any]]
    query_time_ms: float
    total_vectors_searched: int


class BatchQueryResponse(BaseModel):
    results: List[List[Dict[str, Any]]]
    total_queries: int
    avg_query_time_ms: float


# ---- score formatting (S12) ---------------------------------------------------------------
def format_query_results(metric: str, indices, raw_scores, metadata_list) -> List[Dict[str, Any]]:
    """/vectors/query formatting of ``store.query`` output (api/routes/vectors.py:236-258)."""
    out = []
    for i, (_idx, raw, meta) in enumerate(zip(indices, raw_scores, metadata_list)):
        similarity, distance = 0.0, 0.0
        if metric == "cosine":
            similarity = raw
            distance = 1.0 - similarity
        elif metric == "euclidean":
            distance = raw
            similarity = 1.0 / (1.0 + distance)
        elif metric == "dot_product":
            similarity = raw
            distance = -raw
        out.append({"metadata": meta, "similarity_score": similarity, "distance": distance, "rank": i + 1})
    return out


def format_batch_results(metric: str, batch_results) -> List[List[Dict[str, Any]]]:
    """/vectors/batch_query formatting of ``store.batch_query`` output (:294-317): the second
    tuple element is a distance."""
    formatted = []
    for query_results in batch_results:
        rows = []
        if isinstance(query_results, tuple) and len(query_results) == 3:
            indices, distances, metadata_list = query_results
            for i, (_idx, dist, meta) in enumerate(zip(indices, distances, metadata_list)):
                if metric == "cosine":
                    similarity = max(0, 1.0 - dist)
                elif metric == "euclidean":
                    similarity = 1.0 / (1.0 + dist)
                else:
                    similarity = max(0, -dist)
                rows.append({"metadata": meta, "similarity_score": float(similarity), "distance": float(dist),
                             "rank": i + 1})
        formatted.append(rows)
    return formatted


# ---- auth (security/auth.py:34-76): Bearer key, constant-time compare ------------------------
_bearer = HTTPBearer()
_DEFAULT_API_KEY = "mlx-vector-dev-key-2024"


def verify_api_key(credentials: HTTPAuthorizationCredentials = Security(_bearer)) -> str:
    valid = os.getenv("VECTOR_DB_API_KEY") or _DEFAULT_API_KEY
    if not credentials:
        raise HTTPException(status_code=401, detail="Authorization header required",
                            headers={"WWW-Authenticate": "Bearer"})
    if not secrets.compare_digest(credentials.credentials, valid):
        raise HTTPException(status_code=401, detail="Invalid API key", headers={"WWW-Authenticate": "Bearer"})
    return credentials.credentials


# ---- store manager (api/routes/vectors.py:37-141) --------------------------------------------
class VectorStoreManager:
    def __init__(self, config_factory: Optional[Callable[[str, str], MLXVectorStoreConfig]] = None,
                 base_dir: Optional[str] = None):
        self._stores: Dict[str, MLXVectorStore] = {}
        self._configs: Dict[str, MLXVectorStoreConfig] = {}
        self._executor = ThreadPoolExecutor(max_workers=4)
        self._lock = threading.Lock()
        self.config_factory = config_factory or (lambda user_id, model_id: MLXVectorStoreConfig())
        self.base_dir = base_dir

    def _base(self) -> Path:
        return Path(self.base_dir or os.environ.get("VECTOR_STORE_BASE", "~/.team_mind_data/vector_stores")).expanduser()

    def get_store_key(self, user_id: str, model_id: str) -> str:
        return f"{user_id}_{model_id}"

    async def get_store(self, user_id: str, model_id: str,
                        config: Optional[MLXVectorStoreConfig] = None) -> MLXVectorStore:
        key = self.get_store_key(user_id, model_id)
        if key in self._stores:
            return self._stores[key]

        def create() -> MLXVectorStore:
            with self._lock:  # one store object per key even under concurrent first requests
                if key not in self._stores:
                    cfg = config or self.config_factory(user_id, model_id)
                    self._stores[key] = MLXVectorStore(str(self._base() / user_id / model_id), cfg)
                    self._configs[key] = cfg
                    logger.info("initialised store for %s/%s", user_id, model_id)
                return self._stores[key]

        return await asyncio.get_running_loop().run_in_executor(self._executor, create)

    async def delete_store(self, user_id: str, model_id: str) -> Dict[str, Any]:
        key = self.get_store_key(user_id, model_id)
        if key not in self._stores:
            raise ValueError(f"Store not found: {user_id}/{model_id}")
        self._stores.pop(key).clear()
        self._configs.pop(key, None)
        return {"success": True, "message": f"Store {user_id}/{model_id} deleted"}

    async def warmup_all_stores(self):
        loop = asyncio.get_running_loop()
        for key, store in list(self._stores.items()):
            try:
                await loop.run_in_executor(self._executor, store._warmup_kernels)
            except Exception as e:  # the reference logs and continues (:118-119)
                logger.warning("warmup failed for %s: %s", key, e)

    def get_stats(self) -> Dict[str, Any]:
        total_vectors, total_memory = 0, 0.0
        for store in self._stores.values():
            try:
                st = store.get_stats()
                total_vectors += st.get("vector_count", 0)
                total_memory += st.get("memory_usage_mb", 0)
            except Exception as e:
                logger.warning("failed to get stats from store: %s", e)
        return {"total_stores": len(self._stores), "total_vectors": total_vectors,
                "total_memory_mb": total_memory, "mlx_optimized": True, "unified_memory": False}


def create_router(manager: Optional[VectorStoreManager] = None, auth: Callable = verify_api_key) -> APIRouter:
    """The /vectors router over `manager` (a fresh VectorStoreManager by default)."""
    mgr = manager or VectorStoreManager()
    router = APIRouter(prefix="/vectors", tags=["vectors"])
    router.store_manager = mgr  # type: ignore[attr-defined]

    @router.post("/add", response_model=VectorAddResponse)
    async def add_vectors(request: VectorAddRequest, api_key: str = Depends(auth)):
        t0 = time.time()
        try:
            store = await mgr.get_store(request.user_id, request.model_id)
            if not request.vectors or not request.metadata:
                raise HTTPException(status_code=400, detail="Vectors and metadata required")
            import numpy as np
            vectors_np = np.array(request.vectors, dtype=np.float32)
            loop = asyncio.get_running_loop()
            await loop.run_in_executor(mgr._executor, lambda: store.add_vectors(vectors_np, request.metadata))
            return VectorAddResponse(success=True, vectors_added=len(request.vectors),
                                     total_vectors=store.get_stats().get("vector_count", 0),
                                     processing_time_ms=(time.time() - t0) * 1000)
        except Exception as e:  # the reference turns every error, its own 400s included, into a 500
            logger.error("Error adding vectors: %s", e)
            raise HTTPException(status_code=500, detail=f"Failed to add vectors: {e}")

    @router.post("/query", response_model=VectorQueryResponse)
    async def query_vectors(request: VectorQuery, api_key: str = Depends(auth)):
        t0 = time.time()
        try:
            store = await mgr.get_store(request.user_id, request.model_id)
            if not request.query:
                raise HTTPException(status_code=400, detail="Query vector required")
            loop = asyncio.get_running_loop()
            indices, scores, metas = await loop.run_in_executor(
                mgr._executor, lambda: store.query(request.query, k=request.k,
                                                   filter_metadata=request.filter_metadata))
            return VectorQueryResponse(results=format_query_results(store.config.metric, indices, scores, metas),
                                       query_time_ms=(time.time() - t0) * 1000,
                                       total_vectors_searched=store.get_stats().get("vector_count", 0))
        except Exception as e:  # the reference turns every error, its own 400s included, into a 500
            logger.error("Error querying vectors: %s", e, exc_info=True)
            raise HTTPException(status_code=500, detail=f"Query failed: {e}")

    @router.post("/batch_query", response_model=BatchQueryResponse)
    async def batch_query_vectors(request: BatchQueryRequest, api_key: str = Depends(auth)):
        t0 = time.time()
        try:
            store = await mgr.get_store(request.user_id, request.model_id)
            if not request.queries:
                raise HTTPException(status_code=400, detail="Query vectors required")
            loop = asyncio.get_running_loop()
            batch = await loop.run_in_executor(mgr._executor,
                                               lambda: store.batch_query(request.queries, k=request.k))
            total = (time.time() - t0) * 1000
            return BatchQueryResponse(results=format_batch_results(store.config.metric, batch),
                                      total_queries=len(request.queries),
                                      avg_query_time_ms=total / len(request.queries))
        except Exception as e:  # the reference turns every error, its own 400s included, into a 500
            logger.error("Error in batch query: %s", e)
            raise HTTPException(status_code=500, detail=f"Batch query failed: {e}")

    @router.get("/count")
    async def get_vector_count(user_id: str, model_id: str, api_key: str = Depends(auth)):
        try:
            store = await mgr.get_store(user_id, model_id)
            return {"count": store.get_stats().get("vector_count", 0)}
        except Exception as e:
            raise HTTPException(status_code=500, detail=str(e))

    @router.get("/stats")
    async def get_store_stats(user_id: str, model_id: str, api_key: str = Depends(auth)):
        try:
            store = await mgr.get_store(user_id, model_id)
            return {"store_stats": store.get_stats(),
                    "performance_info": {"mlx_optimized": True, "expected_qps": "800-1500",
                                         "target_latency": "<10ms"}}
        except Exception as e:
            raise HTTPException(status_code=500, detail=str(e))

    @router.get("/health")
    async def health_check():
        try:
            g = mgr.get_stats()
            return {"status": "healthy", "mlx_optimized": True, "stores_active": g["total_stores"],
                    "total_vectors": g["total_vectors"], "memory_usage_mb": g["total_memory_mb"]}
        except Exception as e:
            return {"status": "unhealthy", "error": str(e)}

    return router


def create_app(manager: Optional[VectorStoreManager] = None, auth: Callable = verify_api_key):
    """A FastAPI app serving only the /vectors routes (main.py:205 mounts the same router)."""
    from fastapi import FastAPI
    app = FastAPI(title="MLX Vector DB (MI355X core)")
    app.include_router(create_router(manager, auth))
    return app


# module-level router like the reference's (main.py imports `router` from this module)
store_manager = VectorStoreManager()
router = create_router(store_manager)
